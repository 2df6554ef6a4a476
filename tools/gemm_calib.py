"""Calibration: our GEMM variants vs the vendor library (torch.addmm -> hipBLASLt) on the
ViT-MSN batch-256 shapes, interleaved in one process.  The vendor leg is only a yardstick
for what the chip sustains on these shapes; it is never on the product path."""
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


def timeit(fn, n=10):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n


res = {}
for name, (N, K, epi) in shapes.items():
    Mp = (M + 255) // 256 * 256
    A = (torch.randn(Mp, K, device=dev) * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    bb = b.to(torch.bfloat16)
    out = torch.zeros(Mp, N, device=dev) if epi == 2 else torch.zeros(Mp, N, device=dev, dtype=torch.bfloat16)
    s = torch.cuda.current_stream().cuda_stream
    Am = A[:M]
    legs = {}
    for v in variants:
        legs[f"rc{v}"] = (lambda v=v: L.check(lib.rc_gemm_bf16(epi, v, A.data_ptr(), W.data_ptr(), b.data_ptr(), M, N, K,
                                                               out.data_ptr(), None, 0, s)))
    legs["blaslt_addmm"] = lambda: torch.addmm(bb, Am, W.t())
    legs["blaslt_mm"] = lambda: torch.mm(Am, W.t())
    if epi == 1:
        legs["blaslt_addmm+gelu"] = lambda: torch.nn.functional.gelu(torch.addmm(bb, Am, W.t()))
    times = {k: [] for k in legs}
    for r in range(rounds):
        for k, fn in legs.items():
            times[k].append(timeit(fn))
    flops = 2.0 * M * N * K
    res[name] = {k: {"ms_min": min(t), "TFLOPs": flops / (min(t) / 1e3) / 1e12} for k, t in times.items()}
    print(name, json.dumps(res[name]), flush=True)
print(json.dumps(res))
