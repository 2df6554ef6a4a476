"""Where the batch-1 search request's time goes (diagnostic): the bench's
retriever.utils.search over 10k x 768 f32 rows, split into the library call
(rc_sharded_query_host), Index.query, and the reference-shaped search()."""
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = "end-to-end-image-retrieval-service-with-k8s-jenkins_amd"
ing = importlib.import_module(f"{PKG}.ingesting.utils")
ret = importlib.import_module(f"{PKG}.retriever.utils")


def lat(fn, reps=400):
    for _ in range(20):
        fn()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    t = np.array(t) * 1e3
    return {"p50_ms": round(float(np.median(t)), 4), "p99_ms": round(float(np.percentile(t, 99)), 4)}


rng = np.random.default_rng(7)
X = rng.standard_normal((10000, 768)).astype(np.float32)
vec = X[1234].tolist()
ix = ing.get_index("lat-probe", dimension=768, dtype="float32", capacity=len(X))
ix.upsert_tensor([f"r{i}" for i in range(len(X))], torch.from_numpy(X).cuda(), None)
q = np.ascontiguousarray(np.asarray(vec, np.float32)[None])
ss = ix._set
out = {
    "lib_values": lat(lambda: ss.query_host(q, 5, len(X), True)),
    "lib_novalues": lat(lambda: ss.query_host(q, 5, len(X), False)),
    "index_query_values": lat(lambda: ix.query(vector=vec, top_k=5, include_values=True)),
    "index_query_novalues": lat(lambda: ix.query(vector=vec, top_k=5)),
    "search": lat(lambda: ret.search(ix, vec, top_k=5)),
    "asarray": lat(lambda: np.asarray(vec, np.float32)),
}
print(json.dumps(out), flush=True)
