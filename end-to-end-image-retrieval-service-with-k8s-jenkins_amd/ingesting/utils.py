"""Ingest helpers on the MI355X core (mirror of reference ``ingesting/utils.py``).

* ``get_index(index_name)`` — reference ``:23-38`` opens or creates a Pinecone
  cosine index of ``dimension=Config.INPUT_RESOLUTION``; here it opens or creates
  the in-HBM exact index (one per name per process), same ``upsert``/``query``/
  ``fetch`` shapes.
* ``get_feature_vector(image_bytes)`` — reference ``:41-56``: POST the bytes to
  ``Config.EMBEDDING_SERVICE_URL`` as field ``file``; any failure becomes
  ``HTTPException(500, "Failed to get feature vector from embedding service")``.
* ``embed_locally(image_bytes)`` — the same vector computed in-process on the GPU
  (no HTTP hop) for deployments that co-locate ingest with the model.

``get_storage_client`` (GCS) is out of scope: blob storage is not on the hot path.
"""
from __future__ import annotations

import logging
import threading

import requests
from fastapi import HTTPException

from ..config import Config

logger = logging.getLogger(__name__)

_indexes: dict = {}
_lock = threading.Lock()


def index_devices(spec: str | None = None, shards: int | None = None) -> list:
    """Shard placement for ``get_index``: "all" = one shard per visible GPU, "0,2,4" = those
    GPUs, "" = ``shards`` shards on the current GPU."""
    import torch

    spec = Config.INDEX_DEVICES if spec is None else spec
    if spec.strip() == "all":
        return list(range(torch.cuda.device_count()))
    if spec.strip():
        return [int(x) for x in spec.split(",") if x.strip()]
    return [None] * int(shards or Config.INDEX_SHARDS)


def get_index(index_name: str, dimension: int | None = None, dtype: str | None = None, capacity: int | None = None,
              devices: list | None = None):
    """Open or create the named index (reference ``:23-38``): one logical cosine index of
    ``Config.INPUT_RESOLUTION`` dims, row-sharded over ``devices`` (default: ``Config.INDEX_DEVICES``)."""
    from ..index import Index

    with _lock:
        idx = _indexes.get(index_name)
        if idx is None:
            idx = Index(index_name, dimension=dimension or Config.INPUT_RESOLUTION, metric="cosine",
                        dtype=dtype or Config.INDEX_DTYPE, capacity=capacity or Config.INDEX_CAPACITY,
                        devices=devices if devices is not None else index_devices(), filter=Config.INDEX_FILTER)
            _indexes[index_name] = idx
            logger.info("Created in-HBM index: %s", index_name)
        return idx


def get_feature_vector(image_bytes: bytes) -> list:
    try:
        logger.info("Calling embedding service at %s", Config.EMBEDDING_SERVICE_URL)
        response = requests.post(
            url=Config.EMBEDDING_SERVICE_URL,
            files={"file": ("image.jpg", image_bytes, "image/jpeg")},
        )
        response.raise_for_status()
        return response.json()
    except Exception as e:
        logger.error("Failed to get feature vector: %s", e)
        raise HTTPException(status_code=500, detail="Failed to get feature vector from embedding service")


def embed_locally(image_bytes: bytes) -> list:
    from ..embedding.main import embed_bytes

    return embed_bytes(image_bytes)


# embed_bytes validates the upload as the reference's routes do before embedding (embedding/main.py:
# decode_many: UnidentifiedImageError -> 400 "Uploaded file is not a valid image." before the model;
# a stream the GPU decoder rejects goes to PIL, whose other errors propagate as 500), so
# /search_image need not decode it on the host first (retriever/main.py:111-117 does, because its
# embed is a remote call)
embed_locally.validates_image = True
