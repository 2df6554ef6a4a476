"""Oracle (test infrastructure): deterministic seeded ViT-MSN-base weights.

The reference loads ``facebook/vit-msn-base`` by name from the HF hub at import
(``embedding/main.py:33-38``); that checkpoint is not available offline, so
parity runs on weights this module generates from a seed (numpy PCG64).  Keys
follow the checkpoint's legacy layout (transformers 4.46.3, pinned at reference
``requirements.txt:5``): ``encoder.layer.N.attention.attention.query`` etc.
``to_hf_v5`` maps them onto transformers 5.x module names for the golden
generator.
"""
from __future__ import annotations

import numpy as np

HIDDEN = 768
LAYERS = 12
HEADS = 12
MLP = 3072
PATCH = 16
IMAGE = 224
TOKENS = (IMAGE // PATCH) ** 2 + 1  # 197


def vit_msn_shapes(num_layers: int = LAYERS):
    """Ordered (name, shape) list of the ViTMSNModel state dict (legacy key layout)."""
    s = [
        ("embeddings.cls_token", (1, 1, HIDDEN)),
        ("embeddings.position_embeddings", (1, TOKENS, HIDDEN)),
        ("embeddings.patch_embeddings.projection.weight", (HIDDEN, 3, PATCH, PATCH)),
        ("embeddings.patch_embeddings.projection.bias", (HIDDEN,)),
    ]
    for i in range(num_layers):
        p = f"encoder.layer.{i}."
        for nm in ("query", "key", "value"):
            s.append((p + f"attention.attention.{nm}.weight", (HIDDEN, HIDDEN)))
            s.append((p + f"attention.attention.{nm}.bias", (HIDDEN,)))
        s += [
            (p + "attention.output.dense.weight", (HIDDEN, HIDDEN)),
            (p + "attention.output.dense.bias", (HIDDEN,)),
            (p + "intermediate.dense.weight", (MLP, HIDDEN)),
            (p + "intermediate.dense.bias", (MLP,)),
            (p + "output.dense.weight", (HIDDEN, MLP)),
            (p + "output.dense.bias", (HIDDEN,)),
            (p + "layernorm_before.weight", (HIDDEN,)),
            (p + "layernorm_before.bias", (HIDDEN,)),
            (p + "layernorm_after.weight", (HIDDEN,)),
            (p + "layernorm_after.bias", (HIDDEN,)),
        ]
    s += [("layernorm.weight", (HIDDEN,)), ("layernorm.bias", (HIDDEN,))]
    return s


def _std_for(name: str) -> tuple[float, float]:
    """(mean, std) per tensor family — large enough that attention is not uniform."""
    if name.endswith("layernorm_before.weight") or name.endswith("layernorm_after.weight") or name == "layernorm.weight":
        return 1.0, 0.1
    if "layernorm" in name:
        return 0.0, 0.05
    if name.endswith(("query.weight", "key.weight")):
        return 0.0, 0.06
    if name.endswith(".weight"):
        return 0.0, 0.02
    return 0.0, 0.02  # biases, cls token, position embeddings


def seeded_vit_msn_weights(seed: int = 1907, num_layers: int = LAYERS) -> dict[str, np.ndarray]:
    rng = np.random.Generator(np.random.PCG64(seed))
    out = {}
    for name, shape in vit_msn_shapes(num_layers):
        mean, std = _std_for(name)
        out[name] = (rng.standard_normal(shape, dtype=np.float32) * np.float32(std) + np.float32(mean)).astype(np.float32)
    return out


def with_massive_activations(sd: dict[str, np.ndarray], channels=(17, 401), patch_bias: float = 40.0,
                             fc2_bias: float = 20.0, ln_gamma: float = 0.05) -> dict[str, np.ndarray]:
    """A copy of ``sd`` whose residual stream carries trained-ViT-like outlier channels.

    Trained ViTs keep a few hidden channels at ~100x the magnitude of the rest on every
    token ("massive activations"), and their LayerNorm gammas damp those channels.  The
    seeded weights above have no such channels, so they do not stress the bf16 residual
    copy or the LayerNorm fold (rstd·(x·W′ − μ·c), where μ and rstd are then set by the
    outliers).  Here the patch-embedding bias and every layer's fc2 bias push ``channels``
    up (≈ patch_bias + layer·fc2_bias: 280 after 12 layers, against |x| ≈ 1 elsewhere)
    and every LayerNorm gamma of those channels is ``ln_gamma``.
    """
    out = {k: v.copy() for k, v in sd.items()}
    ch = np.asarray(channels)
    out["embeddings.patch_embeddings.projection.bias"][ch] += np.float32(patch_bias)
    for k in out:
        if k.endswith("output.dense.bias") and "attention" not in k:
            out[k][ch] += np.float32(fc2_bias)
        if k.endswith(("layernorm_before.weight", "layernorm_after.weight")) or k == "layernorm.weight":
            out[k][ch] = np.float32(ln_gamma)
    return out


def to_hf_v5(sd: dict[str, np.ndarray]) -> dict[str, np.ndarray]:
    """Legacy checkpoint keys → transformers 5.x ``ViTMSNModel`` module names."""
    ren = {
        "attention.attention.query": "attention.q_proj",
        "attention.attention.key": "attention.k_proj",
        "attention.attention.value": "attention.v_proj",
        "attention.output.dense": "attention.o_proj",
        "intermediate.dense": "mlp.fc1",
        "output.dense": "mlp.fc2",
    }
    out = {}
    for k, v in sd.items():
        nk = k.replace("encoder.layer.", "layers.")
        for a, b in ren.items():
            nk = nk.replace(a, b)
        out[nk] = v
    return out
