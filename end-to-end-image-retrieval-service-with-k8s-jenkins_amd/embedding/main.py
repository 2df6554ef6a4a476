"""``/embed`` service on the MI355X core (mirror of reference ``embedding/main.py``).

Contract kept from the reference (``embedding/main.py:78-124``):
  GET  /         → {"message": "Welcome to ViT-MSN Embedding API. Visit /docs to test."}
  GET  /healthz  → {"status": "healthy"}
  POST /embed    multipart field ``file`` → JSON list[float] (raw CLS vector, 768)
                 400 {"detail": "Uploaded file is not a valid image."} on an unidentifiable image
                 422 when ``file`` is missing; other decode errors propagate (500)

Compute: baseline JPEGs are decoded on the GPU (host Huffman + HIP IDCT /
upsampling / colour, bit-exact with the reference's PIL decode at ``:97``); any
other image goes through PIL on the host as in the reference.  Then one
``rc_embed`` call on the GPU (resize → normalize → ViT-MSN → final LN of the CLS
row) instead of ``extractor`` + ``model`` (``:107-113``).  ``POST /embed_batch`` (field ``files``,
repeated) returns one vector per image — the batched form of the same contract.
OpenTelemetry/Prometheus instrumentation of the reference is out of scope.
"""
from __future__ import annotations

import threading
from io import BytesIO
from typing import List

from fastapi import FastAPI, HTTPException, Request
from fastapi.exceptions import RequestValidationError
from PIL import Image, UnidentifiedImageError

from ..config import Config
from ..multipart import parse_form

app = FastAPI(title="ViT-MSN Embedding Service")

_embedder = None
_embedder_lock = threading.Lock()


def get_embedder():
    """Process-wide model singleton (reference loads it at import, ``:37-39``; here on first use)."""
    global _embedder
    with _embedder_lock:
        if _embedder is None:
            from ..vit import VitMsnEmbedder, random_state_dict

            if Config.MODEL_PATH:
                _embedder = VitMsnEmbedder.from_pretrained(Config.MODEL_PATH, max_batch=Config.EMBED_MAX_BATCH)
            else:  # no checkpoint offline: deterministic seeded weights
                _embedder = VitMsnEmbedder(random_state_dict(Config.WEIGHT_SEED), max_batch=Config.EMBED_MAX_BATCH)
        return _embedder


def _missing_file(field: str):
    return RequestValidationError([{"type": "missing", "loc": ("body", field), "msg": "Field required", "input": None}])


def decode_image(data: bytes) -> Image.Image:
    try:
        return Image.open(BytesIO(data)).convert("RGB")
    except UnidentifiedImageError:
        raise HTTPException(status_code=400, detail="Uploaded file is not a valid image.")


def _gpu_jpeg(data: bytes) -> bool:
    if not Config.GPU_JPEG:
        return False
    from ..jpeg import is_gpu_decodable

    return is_gpu_decodable(data)


def decode_many(blobs: List[bytes]) -> list:
    """Image bytes → u8 HWC RGB images, validated as the reference validates them: baseline
    JPEGs decoded on the GPU (device tensors, bit-exact with PIL), anything else — and any
    stream the GPU decoder rejects — through PIL on the host (``UnidentifiedImageError`` → 400)."""
    import numpy as np

    out: list = [None] * len(blobs)
    gpu = [i for i, b in enumerate(blobs) if _gpu_jpeg(b)]
    gset = set(gpu)
    host = [i for i in range(len(blobs)) if i not in gset]
    for i in host:  # validate before touching the model (400 needs no GPU)
        out[i] = np.asarray(decode_image(blobs[i]), dtype=np.uint8)
    if gpu:
        try:
            for i, im in zip(gpu, get_embedder().decode_jpeg([blobs[i] for i in gpu])):
                out[i] = im
        except ValueError:  # a damaged stream: the reference's host decode decides (image or 400)
            for i in gpu:
                out[i] = np.asarray(decode_image(blobs[i]), dtype=np.uint8)
    return out


def embed_many_device(blobs: List[bytes], normalized: bool = False):
    """Image bytes → (raw [n,768], normed or None) device tensors (the batched ingest path)."""
    images = decode_many(blobs)
    return get_embedder().embed_images(images, normalized=normalized)


def embed_many(blobs: List[bytes]) -> list[list[float]]:
    """Image bytes → raw CLS vectors: GPU JPEG decode where it applies, PIL otherwise."""
    raw, _ = embed_many_device(blobs)
    return raw.cpu().tolist()


def embed_bytes(data: bytes) -> list[float]:
    """Core of /embed: image bytes → raw CLS vector (list of floats)."""
    return embed_many([data])[0]


@app.get("/")
def read_root():
    return {"message": "Welcome to ViT-MSN Embedding API. Visit /docs to test."}


@app.get("/healthz")
def health_check():
    return {"status": "healthy"}


@app.post("/embed", response_model=List[float])
async def embed_image(request: Request):
    form = parse_form(await request.body(), request.headers.get("content-type", ""))
    f = form.get("file")
    if f is None:
        raise _missing_file("file")
    return embed_bytes(f.data)


@app.post("/embed_batch", response_model=List[List[float]])
async def embed_images(request: Request):
    body = await request.body()
    ctype = request.headers.get("content-type", "")
    from email.parser import BytesParser
    from email.policy import HTTP

    if not ctype.lower().startswith("multipart/form-data"):
        raise _missing_file("files")
    msg = BytesParser(policy=HTTP).parsebytes(b"Content-Type: " + ctype.encode("latin-1") + b"\r\n\r\n" + body)
    blobs = [p.get_payload(decode=True) or b"" for p in msg.iter_parts()
             if p.get_param("name", header="content-disposition") == "files"]
    if not blobs:
        raise _missing_file("files")
    return embed_many(blobs)
