"""Embedding precision probe (GPU): 1 - cos(GPU, fp32 oracle) per image for the seeded
weights and for the same weights with trained-ViT-like massive-activation channels
(oracle.weights.with_massive_activations), LayerNorm fold on and off.

    python tools/precision_probe.py [--images N]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch
from PIL import Image

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import import_pkg  # noqa: E402
from oracle.preprocess import preprocess  # noqa: E402
from oracle.vit import cosine, embed_cls  # noqa: E402
from oracle.weights import seeded_vit_msn_weights, with_massive_activations  # noqa: E402


OUTLIERS = (17, 401)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=8)
    a = ap.parse_args()
    vit = import_pkg("vit")
    rng = np.random.default_rng(5)
    imgs = rng.integers(0, 256, (a.images, 224, 224, 3), dtype=np.uint8)
    test = np.array(Image.open(os.path.join(REPO, "tests", "golden", "test_image.jpeg")).convert("RGB").resize((224, 224)))
    imgs[0] = test
    base = seeded_vit_msn_weights(1907)
    res = {}
    for wname, sd in (("seeded", base), ("massive", with_massive_activations(base, channels=OUTLIERS))):
        ref = embed_cls(np.stack([preprocess(x) for x in imgs]), sd)
        m = vit.VitMsnEmbedder(sd, device=0, max_batch=a.images)
        for fold in (True, False):
            m.set_ln_fold(fold)
            raw, _ = m.embed(torch.from_numpy(imgs))
            got = raw.cpu().numpy()
            # distance on the channels other than the outliers (these dominate the norm otherwise)
            keep = np.ones(got.shape[1], bool)
            if wname == "massive":
                keep[list(OUTLIERS)] = False
            d = [float(1.0 - cosine(got[i][keep], ref[i][keep])) for i in range(a.images)]
            res[f"{wname}_fold{int(fold)}"] = {"max": max(d), "median": float(np.median(d)), "all": d}
            print(wname, "fold" if fold else "plain", "max", f"{max(d):.3e}", "median", f"{np.median(d):.3e}", flush=True)
        m.close()
    print(json.dumps({k: {"max": v["max"], "median": v["median"]} for k, v in res.items()}))


if __name__ == "__main__":
    main()
