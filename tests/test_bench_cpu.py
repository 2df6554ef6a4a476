"""bench.py's CPU pieces: the torch-CPU baseline computes the same model as the oracle, and
the multi-GPU launcher hands --gpus N to N ranks (dry run on CPU, gloo)."""
import os
import subprocess
import sys

import numpy as np

from conftest import REPO


def test_torch_baseline_forward_matches_oracle():
    import torch

    sys.path.insert(0, REPO)
    import bench
    from oracle.preprocess import preprocess
    from oracle.vit import cosine, embed_cls
    from oracle.weights import seeded_vit_msn_weights

    sd_np = seeded_vit_msn_weights(0)
    sd = {k: torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32)) for k, v in sd_np.items()}
    imgs = np.random.default_rng(0).integers(0, 256, (2, 224, 224, 3), dtype=np.uint8)
    with torch.inference_mode():
        got = bench.torch_vit_forward(sd)(torch.from_numpy(imgs)).numpy()
    ref = embed_cls(np.stack([preprocess(x) for x in imgs]), sd_np)
    for i in range(2):
        assert 1.0 - cosine(got[i], ref[i]) < 1e-6
        assert np.allclose(got[i], ref[i], atol=2e-3)


def test_bench_gpus_flag_launches_ranks():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    import json

    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2
