"""Run STEPS batch-256 embeds with one GEMM variant and batch-parts setting (a target for
rocprofv3 kernel-trace / PMC passes):  VARIANT=7 PARTS=1 STEPS=5 python tools/embed_run.py"""
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

vit = importlib.import_module("end-to-end-image-retrieval-service-with-k8s-jenkins_amd.vit")
B = int(os.environ.get("BATCH", "256"))
dev = torch.device("cuda", 0)
m = vit.VitMsnEmbedder(vit.random_state_dict(seed=0), device=0, max_batch=B)
m.set_gemm_variant(int(os.environ.get("VARIANT", "0")))
m.set_parts(int(os.environ.get("PARTS", "1")))
g = torch.Generator(device=dev).manual_seed(1)
imgs = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=dev, generator=g)
raw = torch.empty((B, 768), device=dev)
nrm = torch.empty((B, 768), device=dev)
for _ in range(int(os.environ.get("STEPS", "5"))):
    m.embed(imgs, out=(raw, nrm))
torch.cuda.synchronize()
print("ok", float(raw.abs().sum()))
