"""Interleaved A/B of the skinny GEMM's waves per block (diagnostic build, rc_diag_set_skinny_wpb)
on a one-image embed: p50 of the device-side embed time (HIP events around rc_embed, graph replay
on) per setting; the embedding must be the same bits under every setting.
    RC_LIB_PATH=.../lib/diag/libretrieval_core.so python tools/skinny_wpb_ab.py
"""
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

vit = importlib.import_module("end-to-end-image-retrieval-service-with-k8s-jenkins_amd.vit")
_lib = importlib.import_module("end-to-end-image-retrieval-service-with-k8s-jenkins_amd._lib")
lib = _lib.load()
dev = torch.device("cuda", 0)
m = vit.VitMsnEmbedder(vit.random_state_dict(seed=0), device=0, max_batch=4)
g = torch.Generator(device=dev).manual_seed(1)
img = torch.randint(0, 256, (1, 224, 224, 3), dtype=torch.uint8, device=dev, generator=g)
raw, nrm = torch.empty((1, 768), device=dev), torch.empty((1, 768), device=dev)
res, ref = {}, None
for rnd in range(5):
    for wpb in (1, 2, 4):
        _lib.check(lib.rc_diag_set_skinny_wpb(m._h, wpb))
        for _ in range(5):
            m.embed(img, out=(raw, nrm))
        ts = []
        for _ in range(50):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            m.embed(img, out=(raw, nrm))
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        res.setdefault(wpb, []).append(round(ts[len(ts) // 2], 1))
        if ref is None:
            ref = raw.clone()
        assert torch.equal(raw, ref), f"wpb {wpb} changed the embedding bits"
    print(json.dumps({"round": rnd, **{str(k): v[-1] for k, v in res.items()}}), flush=True)
print(json.dumps({"median_us": {str(k): sorted(v)[len(v) // 2] for k, v in res.items()}}))
