"""JPEG streams for the decode tests, encoded here by Pillow (the reference's own
codec, Pillow 12.2.0 / libjpeg-turbo 3.1.4.1): sizes with odd / tiny / non-MCU
dimensions, 4:4:4, 4:2:2, 4:2:0, grayscale, qualities 50-100, restart markers,
plus the reference's fixture image (tests/golden/test_image.jpeg, a copy of the
reference's tests/data/test_image.jpeg)."""
import io
import os

import numpy as np
from PIL import Image

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

SIZES = [(224, 224), (300, 168), (1, 1), (7, 9), (17, 33), (33, 17), (16, 16), (3, 50), (50, 3), (255, 129)]


def synthetic(w: int, h: int, seed: int, mode: str = "RGB", **save_kw) -> bytes:
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (max(h // 4, 1) + 1, max(w // 4, 1) + 1, 3), dtype=np.uint8)
    im = Image.fromarray(base).resize((w, h), Image.BILINEAR)
    arr = np.clip(np.asarray(im).astype(int) + rng.integers(-20, 21, (h, w, 3)), 0, 255).astype(np.uint8)
    im = Image.fromarray(arr)
    if mode == "L":
        im = im.convert("L")
    b = io.BytesIO()
    im.save(b, format="JPEG", **save_kw)
    return b.getvalue()


def cases():
    """[(name, bytes)] of GPU-decodable streams."""
    out = []
    seed = 0
    for (w, h) in SIZES:
        for ss in (0, 1, 2):
            for q in (50, 90, 100):
                seed += 1
                out.append((f"{w}x{h}_ss{ss}_q{q}", synthetic(w, h, seed, quality=q, subsampling=ss)))
        seed += 1
        out.append((f"{w}x{h}_gray", synthetic(w, h, seed, "L", quality=85)))
    out.append(("224_rst3", synthetic(224, 224, 1001, quality=80, subsampling=2, restart_marker_blocks=3)))
    out.append(("101x77_rstrow", synthetic(101, 77, 1002, quality=80, subsampling=1, restart_marker_rows=1)))
    out.append(("test_image", open(os.path.join(GOLDEN, "test_image.jpeg"), "rb").read()))
    return out


def pil_rgb(data: bytes) -> np.ndarray:
    """The reference decode, embedding/main.py:97."""
    return np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
