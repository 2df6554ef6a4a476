"""fc1 (M=50432, N=3072, K=768, GELU epilogue) launched as the product ping-pong
kernel and as its ablations (diagnostic build, tools/build_diag.sh): ABL 8 = no
global stores in the epilogue, ABL 4 = no epilogue, ABL 1 = no DMA in the K loop.
Run under rocprofv3 --pmc (FETCH_SIZE / WRITE_SIZE passes) to see which part of
the kernel causes the HBM reads above the 82 MB of A + W."""
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

L = importlib.import_module("end-to-end-image-retrieval-service-with-k8s-jenkins_amd._lib")
lib = L.load()
dev = torch.device("cuda", 0)
M, N, K = 256 * 197, 3072, 768
Mp = (M + 255) // 256 * 256
A = (torch.randn(Mp, K, device=dev) * 0.5).to(torch.bfloat16)
W = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
b = torch.randn(N, device=dev)
out = torch.zeros(Mp, N, device=dev, dtype=torch.bfloat16)
s = torch.cuda.current_stream().cuda_stream
for v in [int(x) for x in os.environ.get("VARIANTS", "4,108,104,101").split(",")]:
    for _ in range(5):
        L.check(lib.rc_gemm_bf16(1, v, A.data_ptr(), W.data_ptr(), b.data_ptr(), M, N, K, out.data_ptr(), None, 0, s))
    torch.cuda.synchronize()
    print("variant", v, "done", flush=True)
