"""Interleaved A/B of the full-batch projection GEMM kernels inside the real embed (one process).

For each round and each variant: rc_diag_set_gemm_variant (diagnostic build, RC_LIB_PATH), then (a) `steps` timed embeds of a
batch-256 at the bench's --parts (whole-step wall time) and (b) per-GEMM HIP-event timings on
the unsplit batch.  Prints one JSON line per round and a summary (median over rounds).
    python tools/gemm_ab.py [VARIANTS=4,5,6] [ROUNDS=5] [STEPS=10] [ROLES=qkv,oproj,fc1,fc2]
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
variants = [int(v) for v in os.environ.get("VARIANTS", "4,5,6").split(",")]
rounds = int(os.environ.get("ROUNDS", "5"))
steps = int(os.environ.get("STEPS", "10"))
parts = int(os.environ.get("PARTS", "2"))
B = 256
dev = torch.device("cuda", 0)
m = vit.VitMsnEmbedder(vit.random_state_dict(seed=0), device=0, max_batch=B)
g = torch.Generator(device=dev).manual_seed(1)
imgs = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=dev, generator=g)
raw = torch.empty((B, 768), device=dev)
nrm = torch.empty((B, 768), device=dev)
roles = os.environ.get("ROLES", "qkv,oproj,fc1,fc2").split(",")
res = {v: {"step_ms": [], **{r: [] for r in roles}} for v in variants}
ref = None
for r in range(rounds):
    for v in variants:
        m.set_gemm_variant(v)
        m.set_parts(parts)
        for _ in range(2):
            m.embed(imgs, out=(raw, nrm))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            m.embed(imgs, out=(raw, nrm))
        torch.cuda.synchronize()
        res[v]["step_ms"].append((time.perf_counter() - t0) / steps * 1e3)
        if ref is None:
            ref = raw.clone()
        if os.environ.get("NOCHECK") != "1":  # ablation builds change the bits on purpose
            assert torch.equal(raw, ref), f"variant {v} changed the embedding bits"
        m.set_parts(1)
        m.timing(roles)
        m.timing_reset()
        for _ in range(3):
            m.embed(imgs, out=(raw, nrm))
        torch.cuda.synchronize()
        for role in roles:
            ms, n, fl = m.timing_read(role)
            res[v][role].append(ms / max(n, 1) * 1e3)
        m.timing(False)
    print(json.dumps({"round": r, **{str(v): {k: round(x[-1], 2) for k, x in res[v].items()} for v in variants}}), flush=True)
summary = {str(v): {k: round(statistics.median(x), 2) for k, x in res[v].items()} for v in variants}
for v in variants:
    summary[str(v)]["images_per_s"] = round(B / (summary[str(v)]["step_ms"] / 1e3))
print(json.dumps({"summary_median": summary, "units": "step_ms: ms per batch-256 embed at PARTS; GEMMs: us per launch"}))
