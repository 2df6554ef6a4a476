"""Scan lab driver (diagnostic): 1M x 512 f32 rows, stream kernels of tools/scan_lab/lab.hip at
several block counts, interleaved, HIP-event timed; prints GB/s per (variant, blocks) and the
product scan (DeviceIndex.search on the same rows shape) for comparison."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "liblab.so"))
lib.lab_stream.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_void_p]

N, D = 1_000_000, 512
dev = torch.device("cuda:0")
rows = torch.randn((N, D), device=dev)
q = torch.randn(D, device=dev)
out = torch.empty(8192 * 256, device=dev)
names = {0: "U2", 1: "U2_nt", 2: "U1", 3: "U3", 4: "U3_nt"}
cfgs = [(v, b) for v in (0, 1, 2, 3, 4) for b in (1024, 2048, 4096)]
res = {f"{names[v]}_b{b}": [] for v, b in cfgs}
s = torch.cuda.current_stream()
for rnd in range(5):
    for v, b in cfgs:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            assert lib.lab_stream(v, rows.data_ptr(), N, b, q.data_ptr(), out.data_ptr(), ctypes.c_void_p(s.cuda_stream)) == 0
        e1.record()
        torch.cuda.synchronize()
        if rnd > 0:
            res[f"{names[v]}_b{b}"].append(e0.elapsed_time(e1) / 10)
summary = {k: {"us": round(min(t) * 1e3, 1), "GBps": round(N * D * 4 / (min(t) / 1e3) / 1e9, 1)} for k, t in res.items()}
# product scan on the same shape
from importlib import import_module

index = import_module("end-to-end-image-retrieval-service-with-k8s-jenkins_amd.index")
ix = index.DeviceIndex(D, dtype="float32", capacity=N, device=0)
ix.fill_random(2, 0, N)
qq = torch.randn((1, D), device=dev)
for _ in range(5):
    ix.search(qq, 10, N)
torch.cuda.synchronize()
ix.timing(True)
for _ in range(50):
    ix.search(qq, 10, N)
torch.cuda.synchronize()
ms, n, b = ix.timing_read()
summary["product_scan"] = {"us": round(ms / n * 1e3, 1) if n else None, "GBps": round(b / (ms / 1e3) / 1e9, 1) if ms else None}
print(json.dumps(summary), flush=True)
