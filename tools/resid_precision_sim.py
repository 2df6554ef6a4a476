"""CPU simulation: what a plain-bf16 residual stream would cost in embedding precision.

The product keeps the residual stream as a bf16 pair (hi + one byte, ~2^-16 relative); a
plain bf16 stream (2^-9) would halve the residual epilogues' bytes and cut their VALU work.
This restates the GPU arithmetic's roundings in numpy (bf16 GEMM operands and outputs, f32
accumulation, f32 softmax) with the residual stream either kept to 2^-16 ("pair") or rounded
to bf16 ("bf16"), and prints 1 - cos against the fp32 oracle for the seeded weights and the
massive-activation weights (the test bars: 1e-3 fp32 tier, 1e-2 bf16 tier).

    python tools/resid_precision_sim.py [--images N]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle.preprocess import preprocess  # noqa: E402
from oracle.vit import EPS, _gelu, _ln, cosine, embed_cls, patchify  # noqa: E402
from oracle.weights import HEADS, HIDDEN, seeded_vit_msn_weights, with_massive_activations  # noqa: E402


def bf16(x):
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    return r.view(np.float32)


def pair(x):
    """the hi + byte pair: hi = bf16(x), lo = rint((x - hi) / (ulp(hi) / 256))"""
    h = bf16(x)
    e = (h.view(np.uint32) & 0x7F800000).astype(np.int64)
    step = np.where(e >= (16 << 23), ((e - (15 << 23)).astype(np.uint32)).view(np.float32), 0).astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        q = np.where(step > 0, np.clip(np.rint((x - h) / np.where(step > 0, step, 1)), -127, 127), 0)
    return (h + q * step).astype(np.float32)


def mm(a, w):  # bf16 operands, f32 accumulate
    return (bf16(a).astype(np.float64) @ bf16(w).T.astype(np.float64)).astype(np.float32)


def sim_forward(pv, sd, resid):
    rs = bf16 if resid == "bf16" else pair
    B = pv.shape[0]
    nl = sum(1 for k in sd if k.endswith("layernorm_before.weight"))
    wp = sd["embeddings.patch_embeddings.projection.weight"].reshape(HIDDEN, -1)
    x = mm(patchify(pv.astype(np.float32)), wp) + sd["embeddings.patch_embeddings.projection.bias"]
    cls = np.broadcast_to(sd["embeddings.cls_token"], (B, 1, HIDDEN))
    x = rs((np.concatenate([cls, x], axis=1) + sd["embeddings.position_embeddings"]).astype(np.float32))
    S, hd = x.shape[1], HIDDEN // HEADS
    for i in range(nl):
        g = lambda n: sd[f"encoder.layer.{i}." + n]  # noqa: E731
        h = _ln(x, g("layernorm_before.weight"), g("layernorm_before.bias"))
        qkv = [bf16(mm(h, g(f"attention.attention.{n}.weight")) + g(f"attention.attention.{n}.bias"))
               .reshape(B, S, HEADS, hd).transpose(0, 2, 1, 3) for n in ("query", "key", "value")]
        q, k, v = qkv
        s = (q.astype(np.float64) @ k.transpose(0, 1, 3, 2)).astype(np.float32) * np.float32(hd ** -0.5)
        e = np.exp(s - s.max(-1, keepdims=True))
        p = bf16(e / e.sum(-1, keepdims=True))
        o = bf16((p.astype(np.float64) @ v).astype(np.float32)).transpose(0, 2, 1, 3).reshape(B, S, HIDDEN)
        x = rs(x + (mm(o, g("attention.output.dense.weight")) + g("attention.output.dense.bias")))
        h = _ln(x, g("layernorm_after.weight"), g("layernorm_after.bias"))
        h = bf16(_gelu(mm(h, g("intermediate.dense.weight")) + g("intermediate.dense.bias")))
        x = rs(x + (mm(h, g("output.dense.weight")) + g("output.dense.bias")))
    return _ln(x, sd["layernorm.weight"], sd["layernorm.bias"])[:, 0, :]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=4)
    a = ap.parse_args()
    rng = np.random.default_rng(5)
    imgs = rng.integers(0, 256, (a.images, 224, 224, 3), dtype=np.uint8)
    pv = np.stack([preprocess(x) for x in imgs])
    base = seeded_vit_msn_weights(1907)
    outl = (17, 401)
    for wname, sd in (("seeded", base), ("massive", with_massive_activations(base, channels=outl))):
        ref = embed_cls(pv, sd)
        keep = np.ones(HIDDEN, bool)
        if wname == "massive":
            keep[list(outl)] = False
        for resid in ("pair", "bf16"):
            got = sim_forward(pv, sd, resid)
            d = [float(1 - cosine(got[i][keep], ref[i][keep])) for i in range(a.images)]
            dall = [float(1 - cosine(got[i], ref[i])) for i in range(a.images)]
            print(f"{wname:8s} {resid:5s} max 1-cos {max(d):.3e} (all channels {max(dall):.3e})", flush=True)


if __name__ == "__main__":
    main()
