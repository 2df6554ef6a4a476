"""Config 4 per-GPU shard: batched MFMA search timing (rows x 512 fp16, nq queries, top-k)."""
import importlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

M = importlib.import_module("end-to-end-image-retrieval-service-with-k8s-jenkins_amd.index")
n = int(os.environ.get("ROWS", "125000000"))
nq = int(os.environ.get("NQ", "1024"))
k = int(os.environ.get("K", "100"))
reps = int(os.environ.get("REPS", "3"))
d = M.DeviceIndex(512, dtype="float16", capacity=n)
d.fill_random(4, 0, n)
g = torch.Generator(device="cuda").manual_seed(5)
Q = torch.randn((nq, 512), device="cuda", generator=g)
d.search(Q, k, n, mode="mfma")
torch.cuda.synchronize()
d.timing(True)
t = time.perf_counter()
for _ in range(reps):
    d.search(Q, k, n, mode="mfma")
torch.cuda.synchronize()
el = (time.perf_counter() - t) / reps
ms, launches, flops, fb = d.gemm_timing_read()
print(json.dumps({"rows": n, "nq": nq, "k": k, "ms_per_batch": el * 1e3, "queries_per_s": nq / el,
                  "gemm_ms_per_batch": ms / reps, "gemm_launches_per_batch": launches / reps,
                  "gemm_TFLOPs": flops / (ms / 1e3) / 1e12, "fallbacks": fb}), flush=True)
