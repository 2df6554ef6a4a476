"""Tile order of the wide ping-pong GEMMs (QKV, fc1): groups of G row tiles walked column-major
(diagnostic build, rc_diag_set_group_m).  Default: interleaved A/B of G in GROUPS (env, default
"8,4,2,16,0") — step ms at parts = 2 and per-launch QKV / fc1 µs at parts = 1 — with the embedding
bits checked.  --one G: just G, 6 batch-256 embeds at parts = 1 (for rocprofv3 --pmc passes).
    RC_LIB_PATH=.../lib/diag/libretrieval_core.so python tools/group_m_ab.py [--one G]
"""
import importlib
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

vit = importlib.import_module("end-to-end-image-retrieval-service-with-k8s-jenkins_amd.vit")
_lib = importlib.import_module("end-to-end-image-retrieval-service-with-k8s-jenkins_amd._lib")
lib = _lib.load()
B, dev = 256, torch.device("cuda", 0)
m = vit.VitMsnEmbedder(vit.random_state_dict(seed=0), device=0, max_batch=B)
g = torch.Generator(device=dev).manual_seed(1)
imgs = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=dev, generator=g)
raw, nrm = torch.empty((B, 768), device=dev), torch.empty((B, 768), device=dev)
if "--one" in sys.argv:
    _lib.check(lib.rc_diag_set_group_m(m._h, int(sys.argv[sys.argv.index("--one") + 1])))
    m.set_parts(1)
    for _ in range(6):
        m.embed(imgs, out=(raw, nrm))
    torch.cuda.synchronize()
    sys.exit(0)
groups = [int(x) for x in os.environ.get("GROUPS", "8,4,2,16,0").split(",")]
res, ref = {G: {"step_ms": [], "qkv": [], "fc1": []} for G in groups}, None
for rnd in range(4):
    for G in groups:
        _lib.check(lib.rc_diag_set_group_m(m._h, G))
        m.set_parts(2)
        for _ in range(2):
            m.embed(imgs, out=(raw, nrm))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            m.embed(imgs, out=(raw, nrm))
        torch.cuda.synchronize()
        res[G]["step_ms"].append((time.perf_counter() - t0) / 10 * 1e3)
        if ref is None:
            ref = raw.clone()
        assert torch.equal(raw, ref), f"group_m {G} changed the bits"
        m.set_parts(1)
        m.timing(["qkv", "fc1"])
        m.timing_reset()
        for _ in range(3):
            m.embed(imgs, out=(raw, nrm))
        torch.cuda.synchronize()
        for k in ("qkv", "fc1"):
            ms, n, _ = m.timing_read(k)
            res[G][k].append(ms / max(n, 1) * 1e3)
        m.timing(False)
    print(json.dumps({"round": rnd, **{str(G): {k: round(v[-1], 2) for k, v in r.items()} for G, r in res.items()}}), flush=True)
print(json.dumps({"summary_median": {str(G): {k: round(statistics.median(v), 2) for k, v in r.items()} for G, r in res.items()}}))
