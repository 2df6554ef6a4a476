"""Oracle (test infrastructure): ViT-MSN forward in numpy fp32.

Reference: ``embedding/main.py:111-113`` (``model(**inputs)`` then
``last_hidden_state[:, 0, :]``), arithmetic in transformers
``models/vit_msn/modeling_vit_msn.py`` (pinned 4.46.3; container 5.15.0, same math):

* patch embedding ``Conv2d(3, 768, k=16, s=16)`` → flatten → transpose (``:57,66``)
* CLS concat (``:143-144``) + position embeddings (``:154``)
* 12 × pre-LN layer (``:263-283``): ``x + o_proj(attn(LN_before(x)))``,
  ``x + fc2(gelu(fc1(LN_after(x))))``; attention scale ``64**-0.5`` (``:196``),
  softmax in fp32 (``:180``); exact-erf GELU (``activations.py`` ``gelu``)
* final LayerNorm (``:381``), eps 1e-6.
"""
from __future__ import annotations

import numpy as np
from scipy.special import erf

from .weights import HEADS, HIDDEN, PATCH

EPS = 1e-6


def _ln(x, w, b):
    mu = x.mean(-1, keepdims=True, dtype=np.float32)
    var = ((x - mu) ** 2).mean(-1, keepdims=True, dtype=np.float32)
    return ((x - mu) / np.sqrt(var + np.float32(EPS)) * w + b).astype(np.float32)


def _gelu(x):
    return (x * np.float32(0.5) * (np.float32(1.0) + erf(x / np.float32(np.sqrt(2.0))).astype(np.float32))).astype(np.float32)


def patchify(pixel_values: np.ndarray) -> np.ndarray:
    """[B,3,224,224] → [B,196,768] with column index c*256 + kh*16 + kw (the conv weight's K order)."""
    B, C, H, W = pixel_values.shape
    gh, gw = H // PATCH, W // PATCH
    x = pixel_values.reshape(B, C, gh, PATCH, gw, PATCH).transpose(0, 2, 4, 1, 3, 5)
    return np.ascontiguousarray(x.reshape(B, gh * gw, C * PATCH * PATCH))


def vit_msn_forward(pixel_values: np.ndarray, sd: dict, num_layers: int | None = None) -> np.ndarray:
    """[B,3,224,224] f32 → last_hidden_state [B,197,768] f32."""
    B = pixel_values.shape[0]
    if num_layers is None:
        num_layers = sum(1 for k in sd if k.endswith("layernorm_before.weight"))
    wp = sd["embeddings.patch_embeddings.projection.weight"].reshape(HIDDEN, -1)
    x = patchify(pixel_values.astype(np.float32)) @ wp.T + sd["embeddings.patch_embeddings.projection.bias"]
    cls = np.broadcast_to(sd["embeddings.cls_token"], (B, 1, HIDDEN))
    x = np.concatenate([cls, x], axis=1) + sd["embeddings.position_embeddings"]
    x = x.astype(np.float32)
    S = x.shape[1]
    hd = HIDDEN // HEADS
    scale = np.float32(hd ** -0.5)
    for i in range(num_layers):
        p = f"encoder.layer.{i}."
        g = lambda n: sd[p + n]
        h = _ln(x, g("layernorm_before.weight"), g("layernorm_before.bias"))
        q = (h @ g("attention.attention.query.weight").T + g("attention.attention.query.bias")).reshape(B, S, HEADS, hd).transpose(0, 2, 1, 3)
        k = (h @ g("attention.attention.key.weight").T + g("attention.attention.key.bias")).reshape(B, S, HEADS, hd).transpose(0, 2, 1, 3)
        v = (h @ g("attention.attention.value.weight").T + g("attention.attention.value.bias")).reshape(B, S, HEADS, hd).transpose(0, 2, 1, 3)
        s = (q @ k.transpose(0, 1, 3, 2)) * scale
        s = s - s.max(-1, keepdims=True)
        e = np.exp(s)
        pr = (e / e.sum(-1, keepdims=True)).astype(np.float32)
        o = (pr @ v).transpose(0, 2, 1, 3).reshape(B, S, HIDDEN)
        x = (x + (o @ g("attention.output.dense.weight").T + g("attention.output.dense.bias"))).astype(np.float32)
        h = _ln(x, g("layernorm_after.weight"), g("layernorm_after.bias"))
        h = _gelu(h @ g("intermediate.dense.weight").T + g("intermediate.dense.bias"))
        x = (x + (h @ g("output.dense.weight").T + g("output.dense.bias"))).astype(np.float32)
    return _ln(x, sd["layernorm.weight"], sd["layernorm.bias"])


def embed_cls(pixel_values: np.ndarray, sd: dict, num_layers: int | None = None) -> np.ndarray:
    """The /embed output: raw CLS row of the final hidden state, [B,768] (reference main.py:113)."""
    return vit_msn_forward(pixel_values, sd, num_layers)[:, 0, :]


def cosine(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    a = a.astype(np.float64)
    b = b.astype(np.float64)
    return (a * b).sum(-1) / (np.linalg.norm(a, axis=-1) * np.linalg.norm(b, axis=-1))
