"""Interleaved A/B timing of the GEMM tile variants on the ViT-MSN batch-256 shapes (one process)."""
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

L = importlib.import_module("end-to-end-image-retrieval-service-with-k8s-jenkins_amd._lib")
lib = L.load()
dev = torch.device("cuda", 0)
M = 256 * 197
shapes = {"qkv": (2304, 768, 0), "o": (768, 768, 2), "fc1": (3072, 768, 1), "fc2": (768, 3072, 2)}
variants = [int(v) for v in os.environ.get("VARIANTS", "4,8").split(",")]
rounds = int(os.environ.get("ROUNDS", "5"))
res = {}
for name, (N, K, epi) in shapes.items():
    Mp = (M + 255) // 256 * 256
    A = (torch.randn(Mp, K, device=dev) * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    out = torch.zeros(Mp, N, device=dev) if epi == 2 else torch.zeros(Mp, N, device=dev, dtype=torch.bfloat16)
    s = torch.cuda.current_stream().cuda_stream
    times = {v: [] for v in variants}
    for r in range(rounds):
        for v in variants:
            for _ in range(2):
                L.check(lib.rc_gemm_bf16(epi, v, A.data_ptr(), W.data_ptr(), b.data_ptr(), M, N, K, out.data_ptr(), None, 0, s))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                L.check(lib.rc_gemm_bf16(epi, v, A.data_ptr(), W.data_ptr(), b.data_ptr(), M, N, K, out.data_ptr(), None, 0, s))
            e1.record()
            e1.synchronize()
            times[v].append(e0.elapsed_time(e1) / 10)
    flops = 2.0 * M * N * K
    res[name] = {str(v): {"ms_min": min(t), "ms_med": sorted(t)[len(t) // 2], "TFLOPs": flops / (min(t) / 1e3) / 1e12}
                 for v, t in times.items()}
    print(name, json.dumps(res[name]), flush=True)
print(json.dumps(res))
