"""Where batch-1 /embed time goes (diagnostic; run under rocprofv3 --kernel-trace for the device
timeline): embed_bytes on the reference's fixture (tests/data/test_image.jpeg, 300x168), p50 of
the whole call, plus host-side phases timed alone: the Huffman decode to coefficients, the GPU
decode + resize (rc_jpeg_decode_resized), the embed of the already-decoded image (rc_embed +
D2H), and the 768-float list.  --trace-only: just the embed_bytes calls (110), for rocprofv3 --kernel-trace --stats: the
per-kernel totals / 110 are the device time of one request, by kernel."""
import importlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

PKG = "end-to-end-image-retrieval-service-with-k8s-jenkins_amd"
emb = importlib.import_module(f"{PKG}.embedding.main")
J = importlib.import_module(f"{PKG}.jpeg")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
data = open(os.path.join(REPO, "tests", "golden", "test_image.jpeg"), "rb").read()


def lat(fn, reps=100, warm=10):
    for _ in range(warm):
        fn()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append((time.perf_counter() - t0) * 1e3)
    t.sort()
    return {"p50_ms": round(t[len(t) // 2], 4), "min_ms": round(t[0], 4)}


m = emb.get_embedder()
if "--trace-only" in sys.argv:  # for rocprofv3 --stats: 10 warm + 100 embed_bytes calls, nothing else
    r = lat(lambda: emb.embed_bytes(data), reps=100, warm=10)
    print(json.dumps({"embed_bytes": r, "calls": 110}), flush=True)
    sys.exit(0)
out = {}
if hasattr(m, "set_graphs"):  # graph replay of the batch-1 chain vs the stream form, interleaved
    for rnd in range(3):
        for on in (False, True):
            m.set_graphs(on)
            out.setdefault(f"embed_bytes_graphs{int(on)}", []).append(lat(lambda: emb.embed_bytes(data))["p50_ms"])
    m.set_graphs(True)
out["embed_bytes"] = lat(lambda: emb.embed_bytes(data))
dec = m._decoder()
out["huffman_coefficients_host"] = lat(lambda: J.decode_coefficients(data))
out["gpu_decode_resized"] = lat(lambda: (dec.decode_resized([data], 224, 3), torch.cuda.synchronize()))
img = dec.decode_resized([data], 224, 3)
torch.cuda.synchronize()
out["embed_decoded_image"] = lat(lambda: m.embed(img)[0].cpu())
vec = emb.embed_bytes(data)
a = np.asarray(vec, np.float32)
out["tolist_768"] = lat(lambda: a.tolist())
print(json.dumps(out), flush=True)
