"""Oracle (test infrastructure): ViT image preprocessing restated in numpy.

Reference: ``embedding/main.py:107`` ``extractor(images=image, return_tensors="pt")``
→ transformers ``ViTImageProcessor._preprocess`` (``image_processing_backends.py:619-652``):
resize (Pillow, ``oracle.pil_resample``) → ``rescale`` (``image_transforms.py:118-122``:
``u8.astype(f64) * scale`` then ``.astype(f32)``) → ``normalize``
(``image_transforms.py:437``: ``(x - mean_f32) / std_f32`` in f32) → CHW.

The vit-msn-base preprocessor config (resample, mean, std) cannot be read
offline; ``VIT_MSN_PREPROCESS`` records the parameters the build uses (bicubic,
ImageNet mean/std — what the public checkpoint config is believed to carry).
"""
from __future__ import annotations

import numpy as np

from .pil_resample import BICUBIC, resize_u8

IMAGENET_DEFAULT_MEAN = (0.485, 0.456, 0.406)
IMAGENET_DEFAULT_STD = (0.229, 0.224, 0.225)

VIT_MSN_PREPROCESS = {
    "size": (224, 224),
    "resample": BICUBIC,
    "rescale_factor": 1.0 / 255.0,
    "image_mean": IMAGENET_DEFAULT_MEAN,
    "image_std": IMAGENET_DEFAULT_STD,
}


def preprocess(img_hwc_u8: np.ndarray, params: dict = VIT_MSN_PREPROCESS) -> np.ndarray:
    """HxWx3 u8 → [3, 224, 224] f32 pixel_values."""
    oh, ow = params["size"]
    x = resize_u8(img_hwc_u8, oh, ow, params["resample"])
    x = (x.astype(np.float64) * params["rescale_factor"]).astype(np.float32)
    mean = np.array(params["image_mean"], dtype=np.float32)
    std = np.array(params["image_std"], dtype=np.float32)
    x = (x - mean) / std
    return np.ascontiguousarray(x.transpose(2, 0, 1))


def pixel_lut(params: dict = VIT_MSN_PREPROCESS) -> np.ndarray:
    """[3, 256] f32: the exact f32 value ``normalize(rescale(u))`` for every u8 ``u``."""
    u = np.arange(256, dtype=np.uint8)
    x = (u.astype(np.float64) * params["rescale_factor"]).astype(np.float32)
    mean = np.array(params["image_mean"], dtype=np.float32)
    std = np.array(params["image_std"], dtype=np.float32)
    return np.stack([(x - mean[c]) / std[c] for c in range(3)]).astype(np.float32)
