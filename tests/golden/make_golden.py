"""Generate the committed golden vectors under ``tests/golden/``.

Run in the build container (CPU): ``python tests/golden/make_golden.py``.

The reference's arithmetic lives in third-party code that IS importable here:
Pillow 12.2.0 (reference pins ``pillow==10.4.0``, ``requirements.txt:7``) and
transformers 5.15.0 (pins ``transformers==4.46.3``, ``requirements.txt:5``).
The reference modules themselves are not importable (they need pinecone,
google-cloud-storage, opentelemetry, loguru and a by-name hub download at
import — ``embedding/main.py:37-38``), so this script drives the same library
calls the reference makes:

* ``Image.open(BytesIO(bytes)).convert("RGB")``        (``embedding/main.py:97``)
* ``ViTImageProcessor``(PIL backend) ``(images=image)`` (``embedding/main.py:107``)
* ``ViTMSNModel(...)(**inputs).last_hidden_state[:, 0, :]`` (``embedding/main.py:111-113``)

with deterministic seeded weights (``oracle.weights``) because the
``facebook/vit-msn-base`` checkpoint cannot be fetched offline.  The exact
cosine top-k goldens are build-generated (Pinecone stand-in: parity unpinned
beyond the reference's contract tests).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
from io import BytesIO

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle.cosine_topk import cosine_topk, planted_index  # noqa: E402
from oracle.preprocess import VIT_MSN_PREPROCESS  # noqa: E402
from oracle.weights import seeded_vit_msn_weights, to_hf_v5  # noqa: E402

WEIGHT_SEED = 1907
INDEX_ROWS = 10_000
INDEX_DIM = 768
INDEX_SEED = 0


def sha16(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def hf_processor():
    from transformers.models.vit.image_processing_pil_vit import ViTImageProcessorPil

    p = VIT_MSN_PREPROCESS
    return ViTImageProcessorPil(
        size={"height": p["size"][0], "width": p["size"][1]},
        resample=p["resample"],
        image_mean=list(p["image_mean"]),
        image_std=list(p["image_std"]),
        rescale_factor=p["rescale_factor"],
    )


def hf_model(sd, num_layers):
    import torch
    from transformers import ViTMSNConfig, ViTMSNModel

    cfg = ViTMSNConfig(num_hidden_layers=num_layers)
    cfg._attn_implementation = "eager"
    m = ViTMSNModel(cfg).eval()
    missing, unexpected = m.load_state_dict({k: torch.from_numpy(v) for k, v in to_hf_v5(sd).items()}, strict=True)
    assert not missing and not unexpected
    return m


def main():
    import torch
    from PIL import Image

    torch.manual_seed(0)
    out = {}
    with open(os.path.join(HERE, "test_image.jpeg"), "rb") as f:
        jpeg = f.read()
    img = Image.open(BytesIO(jpeg)).convert("RGB")
    arr = np.array(img)
    out["decoded_shape"] = list(arr.shape)
    out["decoded_sha16"] = sha16(arr)
    out["resized_u8_sha16"] = sha16(np.array(img.resize((224, 224), resample=VIT_MSN_PREPROCESS["resample"])))

    proc = hf_processor()
    pv = proc(images=img, return_tensors="np")["pixel_values"][0].astype(np.float32)
    out["pixel_values_sha16"] = sha16(pv)
    out["preprocess"] = {k: (list(v) if isinstance(v, tuple) else v) for k, v in VIT_MSN_PREPROCESS.items()}

    # full 12-layer model, seeded weights
    sd = seeded_vit_msn_weights(WEIGHT_SEED)
    m = hf_model(sd, 12)
    with torch.no_grad():
        emb = m(pixel_values=torch.from_numpy(pv)[None]).last_hidden_state[:, 0, :].numpy()[0]
    np.save(os.path.join(HERE, "test_image_embedding_seed1907.npy"), emb.astype(np.float32))

    # 2-layer model on two synthetic 224x224 images (fast oracle test)
    sd2 = seeded_vit_msn_weights(WEIGHT_SEED, num_layers=2)
    m2 = hf_model(sd2, 2)
    rng = np.random.Generator(np.random.PCG64(1))
    imgs = rng.integers(0, 256, (2, 224, 224, 3), dtype=np.uint8)
    np.save(os.path.join(HERE, "synthetic_u8_2x224.npy"), imgs)
    pv2 = proc(images=[Image.fromarray(x) for x in imgs], return_tensors="np")["pixel_values"].astype(np.float32)
    with torch.no_grad():
        emb2 = m2(pixel_values=torch.from_numpy(pv2)).last_hidden_state[:, 0, :].numpy()
    np.save(os.path.join(HERE, "synthetic_embedding_2layer_seed1907.npy"), emb2.astype(np.float32))

    # exact cosine top-5 over a seeded 10k x 768 index (config 1)
    X, planted = planted_index(emb)
    rows, scores = cosine_topk(X, emb, 5)
    out["index"] = {"rows": INDEX_ROWS, "dim": INDEX_DIM, "seed": INDEX_SEED, "planted": planted}
    out["top5_rows"] = rows[0].tolist()
    out["top5_scores"] = scores[0].tolist()
    out["weight_seed"] = WEIGHT_SEED
    out["generator"] = {"transformers": __import__("transformers").__version__,
                        "pillow": Image.__version__ if hasattr(Image, "__version__") else __import__("PIL").__version__,
                        "torch": torch.__version__}
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
