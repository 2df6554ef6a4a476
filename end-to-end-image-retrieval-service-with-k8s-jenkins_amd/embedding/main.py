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
from ..multipart import parse_form, parse_form_all

app = FastAPI(title="ViT-MSN Embedding Service")

_embedder = None
_embedder_lock = threading.Lock()


def embed_devices(spec: str | None = None) -> list:
    """GPUs of the embedding replicas: ``Config.EMBED_DEVICES`` ("all", "0,1", repeats allowed),
    or by default the distinct GPUs the index shards live on (one model per GPU)."""
    import torch

    spec = Config.EMBED_DEVICES if spec is None else spec
    if spec.strip() == "all":
        return list(range(torch.cuda.device_count()))
    if spec.strip():
        return [int(x) for x in spec.split(",") if x.strip()]
    from ..ingesting.utils import index_devices

    out = []
    for d in index_devices():
        d = torch.cuda.current_device() if d is None else int(d)
        if d not in out:
            out.append(d)
    return out


def get_embedder():
    """Process-wide model singleton (reference loads it at import, ``:37-39``; here on first use).

    One GPU: a ``VitMsnEmbedder``.  Several (``embed_devices()``): an ``EmbedderPool`` with
    one model per GPU — the reference's embedding replicas (``helm_charts/embedding/
    values.yaml:1``) as data parallelism inside the process, no collectives."""
    global _embedder
    with _embedder_lock:
        if _embedder is None:
            from ..vit import EmbedderPool, VitMsnEmbedder, load_checkpoint_dir, random_state_dict

            devs = embed_devices()
            if Config.MODEL_PATH:
                sd, cfg, pre = load_checkpoint_dir(Config.MODEL_PATH)
            else:  # no checkpoint offline: deterministic seeded weights
                sd, cfg, pre = random_state_dict(Config.WEIGHT_SEED), None, None
            if len(devs) > 1:
                _embedder = EmbedderPool(sd, devs, max_batch=Config.EMBED_MAX_BATCH, model_config=cfg, preprocess=pre)
            else:
                _embedder = VitMsnEmbedder(sd, device=devs[0] if devs else None, max_batch=Config.EMBED_MAX_BATCH,
                                           model_config=cfg, preprocess=pre)
        return _embedder


def reset_embedder() -> None:
    """Drop the singleton (tests / reconfiguration); the next get_embedder() builds it anew."""
    global _embedder
    with _embedder_lock:
        if _embedder is not None:
            _embedder.close()
        _embedder = None


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
    """Image bytes → the embedder's u8 HWC RGB inputs, validated as the reference validates
    them: baseline JPEGs decoded AND resized to the model's input size on the GPU in one pass
    (device tensors, bit-exact with PIL decode + the processor's resize), anything else — and
    any stream the GPU decoder rejects — through PIL on the host at its own size
    (``UnidentifiedImageError`` → 400), resized later inside rc_embed."""
    import numpy as np
    import torch

    out: list = [None] * len(blobs)
    gpu = [i for i, b in enumerate(blobs) if _gpu_jpeg(b)]
    gset = set(gpu)
    host = [i for i in range(len(blobs)) if i not in gset]
    for i in host:  # validate before touching the model (400 needs no GPU)
        out[i] = np.asarray(decode_image(blobs[i]), dtype=np.uint8)
    if gpu:
        try:
            ims = get_embedder().decode_jpeg_for_embed([blobs[i] for i in gpu])  # a pool decodes per member GPU
            for i, im in zip(gpu, ims.unbind(0) if isinstance(ims, torch.Tensor) else ims):
                out[i] = im
        except ValueError:  # a damaged stream: the reference's host decode decides (image or 400)
            for i in gpu:
                out[i] = np.asarray(decode_image(blobs[i]), dtype=np.uint8)
    return out


def embed_many_device(blobs: List[bytes], normalized: bool = False):
    """Image bytes → (raw [n,768], normed or None) device tensors (the batched ingest path)."""
    return _embed_decoded(decode_many(blobs), normalized)


def _embed_decoded(images: list, normalized: bool = False):
    emb = get_embedder()
    if hasattr(emb, "assign_by_location"):  # a pool: embed each image on the GPU that decoded it
        return emb.embed_images(images, normalized=normalized, assign=emb.assign_by_location(images))
    return emb.embed_images(images, normalized=normalized)


def embed_many(blobs: List[bytes]) -> list[list[float]]:
    """Image bytes → raw CLS vectors: GPU JPEG decode where it applies, PIL otherwise.  Each
    vector is a list of Python floats (the /embed body) that also carries its float32 row
    (``index.F32List``), for in-process callers that hand it straight to ``index.query``."""
    import torch

    from ..index import F32List

    images = decode_many(blobs)  # validates first: a non-image is a 400 before the model loads
    emb = get_embedder()
    if len(blobs) == 1 and not hasattr(emb, "assign_by_location"):
        # the /embed request: the final kernel writes the vector straight into pinned host memory
        # (no D2H copy), then one stream sync
        host = torch.empty((1, emb.hidden), dtype=torch.float32, pin_memory=True)
        emb.embed_images(images, out=(host, None))
        torch.cuda.current_stream(emb.device).synchronize()
        a = host.numpy().copy()  # 3 KB: the pinned block goes back to torch's pool now, not when
        # the caller drops the embedding (ingest results, caches)
    else:
        raw, _ = _embed_decoded(images)
        a = raw.cpu().numpy()
    return [F32List(row.tolist(), row) for row in a]


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
    files = parse_form_all(await request.body(), request.headers.get("content-type", "")).get("files")
    if not files:
        raise _missing_file("files")
    return embed_many([f.data for f in files])
