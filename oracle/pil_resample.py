"""Oracle (test infrastructure): Pillow ``Image.resize`` restated in numpy.

Reference call site: ``embedding/main.py:107`` → ``ViTImageProcessor`` →
``transformers/image_transforms.py:367`` ``image.resize((w, h), resample=...)``
→ Pillow (pinned ``pillow==10.4.0`` in reference ``requirements.txt:7``;
container has 12.2.0 — the libImaging resample algorithm is unchanged between
them).  Pillow's C source is not in the container, so this restates its
published ``libImaging/Resample.c`` algorithm:

* ``precompute_coeffs``: support scaled by the downscale factor (antialias),
  per-output-pixel window [xmin, xmin+xmax), weights normalised in double;
* ``normalize_coeffs_8bpc``: weights quantised to 22 fractional bits with
  round-half-away-from-zero;
* horizontal pass first (only over the source rows the vertical pass needs),
  u8-clamped intermediate, then the vertical pass; each pass adds the 0.5
  rounding bias ``1 << 21`` and clips ``acc >> 22`` to [0, 255];
* a pass is skipped when its axis size is unchanged; an unchanged image is a
  copy.

Pinned bit-exactly against Pillow 12.2.0 by ``tests/test_oracle_golden.py``.
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2  # 22

BILINEAR = 2  # PIL.Image.Resampling.BILINEAR
BICUBIC = 3   # PIL.Image.Resampling.BICUBIC


def _bicubic(x: float) -> float:
    a = -0.5
    x = abs(x)
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1.0
    if x < 2.0:
        return (((x - 5.0) * x + 8.0) * x - 4.0) * a
    return 0.0


def _bilinear(x: float) -> float:
    x = abs(x)
    if x < 1.0:
        return 1.0 - x
    return 0.0


_FILTERS = {BICUBIC: (_bicubic, 2.0), BILINEAR: (_bilinear, 1.0)}


def precompute_coeffs(in_size: int, out_size: int, resample: int):
    """Return (bounds[out,2] int32, kk[out,ksize] float64, ksize) — Resample.c precompute_coeffs."""
    filt, fsupport = _FILTERS[resample]
    in0, in1 = 0.0, float(in_size)
    scale = (in1 - in0) / out_size
    filterscale = max(scale, 1.0)
    support = fsupport * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), dtype=np.int32)
    kk = np.zeros((out_size, ksize), dtype=np.float64)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = in0 + (xx + 0.5) * scale
        xmin = int(center - support + 0.5)  # C (int) truncation
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        ww = 0.0
        for x in range(xmax):
            w = filt((x + xmin - center + 0.5) * ss)
            kk[xx, x] = w
            ww += w
        if ww != 0.0:
            for x in range(xmax):
                kk[xx, x] /= ww
        bounds[xx] = (xmin, xmax)
    return bounds, kk, ksize


def normalize_coeffs_8bpc(kk: np.ndarray) -> np.ndarray:
    """Fixed-point weights, round half away from zero (C cast truncates)."""
    scaled = kk * float(1 << PRECISION_BITS)
    out = np.where(kk < 0, np.trunc(-0.5 + scaled), np.trunc(0.5 + scaled))
    return out.astype(np.int64)


def _clip8(acc: np.ndarray) -> np.ndarray:
    return np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)


def _pass(src: np.ndarray, bounds, kfix, axis: int) -> np.ndarray:
    """One separable pass along ``axis`` (1 = horizontal, 0 = vertical) of an HxWxC u8 image."""
    out_size, ksize = kfix.shape
    s = src.astype(np.int64)
    if axis == 1:
        acc = np.full((src.shape[0], out_size, src.shape[2]), 1 << (PRECISION_BITS - 1), dtype=np.int64)
        for xx in range(out_size):
            xmin, xmax = bounds[xx]
            acc[:, xx, :] += np.einsum("hkc,k->hc", s[:, xmin:xmin + xmax, :], kfix[xx, :xmax])
    else:
        acc = np.full((out_size, src.shape[1], src.shape[2]), 1 << (PRECISION_BITS - 1), dtype=np.int64)
        for yy in range(out_size):
            ymin, ymax = bounds[yy]
            acc[yy] += np.einsum("kwc,k->wc", s[ymin:ymin + ymax], kfix[yy, :ymax])
    return _clip8(acc)


def resize_u8(img: np.ndarray, out_h: int, out_w: int, resample: int = BICUBIC) -> np.ndarray:
    """Pillow-exact resize of an HxWx3 u8 RGB image (ImagingResampleInner)."""
    assert img.dtype == np.uint8 and img.ndim == 3
    in_h, in_w = img.shape[:2]
    if (in_h, in_w) == (out_h, out_w):
        return img.copy()
    need_h = out_w != in_w
    need_v = out_h != in_h
    bh, kh, _ = precompute_coeffs(in_w, out_w, resample)
    bv, kv, _ = precompute_coeffs(in_h, out_h, resample)
    cur = img
    if need_h:
        y_first = int(bv[0, 0])
        y_last = int(bv[-1, 0] + bv[-1, 1])
        bv = bv.copy()
        bv[:, 0] -= y_first
        cur = _pass(img[y_first:y_last], bh, normalize_coeffs_8bpc(kh), axis=1)
    if need_v:
        cur = _pass(cur, bv, normalize_coeffs_8bpc(kv), axis=0)
    return cur
