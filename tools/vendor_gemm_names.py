"""Run the embedding's four GEMM shapes through torch.mm (hipBLASLt) so that
`rocprofv3 --kernel-trace --stats -- python tools/vendor_gemm_names.py` names the vendor
kernels (their Tensile names carry macro tile, depth-U, prefetch and LDS options) and their
durations — the reference point for csrc/gemm.h's ping-pong kernel.  Diagnostic only."""
import torch

M = 256 * 197
SHAPES = {"qkv": (2304, 768), "o": (768, 768), "fc1": (3072, 768), "fc2": (768, 3072)}
torch.manual_seed(0)
for role, (n, k) in SHAPES.items():
    a = torch.randn(M, k, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
    for _ in range(10):
        c = torch.mm(a, w.t())
    torch.cuda.synchronize()
    print(role, tuple(c.shape), flush=True)
