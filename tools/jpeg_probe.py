"""The fused JPEG decode -> Pillow-exact resize on its own (diagnostic; run under rocprofv3
--kernel-trace --stats for per-kernel times): 256 fixture-shaped (168x300 WxH, the reference's
tests/data/test_image.jpeg shape) q90 4:2:0 JPEGs per call, and single images (the /embed
request: the fixture itself).  Prints host wall time per call (host Huffman + H2D + kernels)."""
import importlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import synthetic_jpegs  # noqa: E402

J = importlib.import_module("end-to-end-image-retrieval-service-with-k8s-jenkins_amd.jpeg")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
fixture = open(os.path.join(REPO, "tests", "golden", "test_image.jpeg"), "rb").read()
batch = synthetic_jpegs(256, 7100, size=(168, 300))
dec = J.JpegDecoder(device=0, max_images=256, max_pixels=256 * 168 * 304)
out = {}
for name, datas, reps in (("fixture_shape_256", batch, 20), ("fixture_1", [fixture], 200)):
    for _ in range(3):
        dec.decode_resized(datas, 224, 3)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        dec.decode_resized(datas, 224, 3)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    ts.sort()
    out[name] = {"p50_ms": round(ts[len(ts) // 2], 4), "min_ms": round(ts[0], 4), "reps": reps, "images": len(datas)}
print(json.dumps(out), flush=True)
