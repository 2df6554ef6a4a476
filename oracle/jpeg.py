"""TEST INFRASTRUCTURE ONLY (oracle): numpy restatement of libjpeg-turbo's default
pixel reconstruction, the arithmetic behind Pillow's ``Image.open(jpeg).convert("RGB")``
(reference ``embedding/main.py:97``).  Third-party algorithm, absent from
/root/reference: libjpeg-turbo 3.1.4.1 as bundled with Pillow 12.2.0 (no C
source in this container); restated from its published algorithms:

* ``idct_islow``     jidctint.c ``jpeg_idct_islow`` (CONST_BITS 13, PASS1_BITS 2),
                     output clamped to [0, 255] after +128 (the SIMD islow's
                     saturating pack; equals the C range-limit table for |x| < 512);
* ``upsample``       jdsample.c fancy upsampling: ``h2v1_fancy_upsample``,
                     ``h1v2_fancy_upsample``, ``h2v2_fancy_upsample`` (context rows
                     replicated at the top/bottom edge, jdmainct.c), plain
                     replication when the downsampled width is <= 2;
* ``ycc_to_rgb``     jdcolor.c ``build_ycc_rgb_table`` / ``ycc_rgb_convert``
                     (SCALEBITS 16, ONE_HALF rounding).

Inputs are the quantised coefficients of the library's host entropy decoder
(``rc_jpeg_decode_coefficients``); tests pin this restatement bit-exact against
Pillow's own decode of the same bytes.  Never imported by the package.
"""
from __future__ import annotations

import numpy as np

C = dict(F0298=2446, F0390=3196, F0541=4433, F0765=6270, F0899=7373, F1175=9633, F1501=12299, F1847=15137,
         F1961=16069, F2053=16819, F2562=20995, F3072=25172)


def _idct_1d(x):
    """x [..., 8] int64 -> 8 undescaled outputs (jidctint.c, one pass)."""
    z2, z3 = x[..., 2], x[..., 6]
    z1 = (z2 + z3) * C["F0541"]
    tmp2 = z1 + z3 * -C["F1847"]
    tmp3 = z1 + z2 * C["F0765"]
    z2, z3 = x[..., 0], x[..., 4]
    tmp0 = (z2 + z3) << 13
    tmp1 = (z2 - z3) << 13
    tmp10, tmp13, tmp11, tmp12 = tmp0 + tmp3, tmp0 - tmp3, tmp1 + tmp2, tmp1 - tmp2
    t0, t1, t2, t3 = x[..., 7], x[..., 5], x[..., 3], x[..., 1]
    z1, z2, z3, z4 = t0 + t3, t1 + t2, t0 + t2, t1 + t3
    z5 = (z3 + z4) * C["F1175"]
    t0, t1, t2, t3 = t0 * C["F0298"], t1 * C["F2053"], t2 * C["F3072"], t3 * C["F1501"]
    z1, z2, z3, z4 = z1 * -C["F0899"], z2 * -C["F2562"], z3 * -C["F1961"], z4 * -C["F0390"]
    z3 = z3 + z5
    z4 = z4 + z5
    t0 = t0 + z1 + z3
    t1 = t1 + z2 + z4
    t2 = t2 + z2 + z3
    t3 = t3 + z1 + z4
    return np.stack([tmp10 + t3, tmp11 + t2, tmp12 + t1, tmp13 + t0, tmp13 - t0, tmp12 - t1, tmp11 - t2, tmp10 - t3],
                    axis=-1)


def _descale(x, n):
    return (x + (1 << (n - 1))) >> n


def idct_islow(coef: np.ndarray, qtab: np.ndarray) -> np.ndarray:
    """coef int16 [nb, 64] natural order, qtab [64] -> u8 samples [nb, 8, 8]."""
    x = coef.astype(np.int64).reshape(-1, 8, 8) * qtab.astype(np.int64).reshape(8, 8)
    ws = _descale(_idct_1d(np.swapaxes(x, 1, 2)), 11)      # columns: [nb, col, row]
    out = _descale(_idct_1d(np.swapaxes(ws, 1, 2)), 18)    # rows:    [nb, row, col]
    return np.clip(out + 128, 0, 255).astype(np.uint8)


def plane_samples(blocks_u8: np.ndarray, bw: int, bh: int) -> np.ndarray:
    """[bh*bw, 8, 8] raster blocks -> [bh*8, bw*8] sample plane."""
    return blocks_u8.reshape(bh, bw, 8, 8).transpose(0, 2, 1, 3).reshape(bh * 8, bw * 8)


def upsample(p: np.ndarray, rx: int, ry: int, dw: int, dh: int, W: int, H: int) -> np.ndarray:
    """Downsampled plane (real size dh x dw, padded allowed) -> H x W (jdsample.c)."""
    p = p[:dh, :dw].astype(np.int32)
    if rx == 1 and ry == 1:
        return p[:H, :W]
    if ry == 1:  # h2v1
        if dw <= 2:
            return np.repeat(p, 2, axis=1)[:H, :W]
        left = np.concatenate([p[:, :1], p[:, :-1]], axis=1)
        right = np.concatenate([p[:, 1:], p[:, -1:]], axis=1)
        even = (3 * p + left + 1) >> 2
        odd = (3 * p + right + 2) >> 2
        even[:, 0] = p[:, 0]
        odd[:, -1] = p[:, -1]
        out = np.stack([even, odd], axis=2).reshape(dh, 2 * dw)
        return out[:H, :W]
    above = np.concatenate([p[:1], p[:-1]], axis=0)
    below = np.concatenate([p[1:], p[-1:]], axis=0)
    if rx == 1:  # h1v2
        top = (3 * p + above + 1) >> 2
        bot = (3 * p + below + 2) >> 2
        return np.stack([top, bot], axis=1).reshape(2 * dh, dw)[:H, :W]
    if dw <= 2:  # h2v2 without context
        return np.repeat(np.repeat(p, 2, axis=0), 2, axis=1)[:H, :W]
    rows = []
    for far in (above, below):
        cs = 3 * p + far
        left = np.concatenate([cs[:, :1], cs[:, :-1]], axis=1)
        right = np.concatenate([cs[:, 1:], cs[:, -1:]], axis=1)
        even = (3 * cs + left + 8) >> 4
        odd = (3 * cs + right + 7) >> 4
        even[:, 0] = (cs[:, 0] * 4 + 8) >> 4
        odd[:, -1] = (cs[:, -1] * 4 + 7) >> 4
        rows.append(np.stack([even, odd], axis=2).reshape(dh, 2 * dw))
    return np.stack(rows, axis=1).reshape(2 * dh, 2 * dw)[:H, :W]


def ycc_to_rgb(Y: np.ndarray, Cb: np.ndarray, Cr: np.ndarray) -> np.ndarray:
    y = Y.astype(np.int64)
    cb = Cb.astype(np.int64) - 128
    cr = Cr.astype(np.int64) - 128
    r = y + ((91881 * cr + 32768) >> 16)
    g = y + ((-22554 * cb + 32768 - 46802 * cr) >> 16)
    b = y + ((116130 * cb + 32768) >> 16)
    return np.clip(np.stack([r, g, b], axis=-1), 0, 255).astype(np.uint8)


def reconstruct(info, coef: np.ndarray, qtab: np.ndarray) -> np.ndarray:
    """(rc_jpeg_info, coefficients, quant tables) -> H x W x 3 u8, as PIL .convert("RGB")."""
    W, H, nc = info.width, info.height, info.ncomp
    planes, b0 = [], 0
    for c in range(nc):
        bw, bh = info.bw[c], info.bh[c]
        blocks = idct_islow(coef[b0:b0 + bw * bh], qtab[c])
        b0 += bw * bh
        rx, ry = info.hmax // info.h[c], info.vmax // info.v[c]
        dw = -(-W * info.h[c] // info.hmax)
        dh = -(-H * info.v[c] // info.vmax)
        planes.append(upsample(plane_samples(blocks, bw, bh), rx, ry, dw, dh, W, H))
    if nc == 1:
        g = planes[0].astype(np.uint8)
        return np.stack([g, g, g], axis=-1)
    return ycc_to_rgb(*planes)
