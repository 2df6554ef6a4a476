"""Save the raw embeddings of 64 seeded images (12-layer seeded model) to gpurun_out/embed_<TAG>.npy,
for bit comparisons between two builds (RC_LIB_PATH selects the library)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import import_pkg  # noqa: E402
from oracle.weights import seeded_vit_msn_weights  # noqa: E402

vit = import_pkg("vit")
imgs = torch.from_numpy(np.random.default_rng(3).integers(0, 256, (64, 224, 224, 3), dtype=np.uint8))
m = vit.VitMsnEmbedder(seeded_vit_msn_weights(1907), device=0, max_batch=64)
r, _ = m.embed(imgs)
os.makedirs("gpurun_out", exist_ok=True)
np.save(f"gpurun_out/embed_{sys.argv[1]}.npy", r.cpu().numpy())
