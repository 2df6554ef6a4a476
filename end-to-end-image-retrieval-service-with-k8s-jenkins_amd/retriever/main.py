"""Retriever service on the MI355X core (mirror of reference ``retriever/main.py``).

Contract kept (``retriever/main.py:94-169``):
  GET  /              → {"message": "Welcome to the Image Retriever API. Visit /docs to test."}
  GET  /healthz       → {"status": "OK!"}
  POST /search_image  multipart ``file`` → list of ≤ TOP_K image URLs, best match first
                      ([] when the index has no match); 400 "Uploaded file is not a valid
                      image."; 422 without ``file``

Flow as in the reference: validation decode (``:111-117``; folded into the in-process embed,
which validates with the same 400 body before the model runs) → ``get_feature_vector``
(``:122``; in process by default, see ingesting.main) → ``search(index, feature,
top_k=Config.TOP_K)`` (``:128``, the HIP exact top-k) → ``index.fetch(ids)``
(``:142``) → one URL per match from its ``gcs_path`` metadata (``:148-168``; the
GCS signing is the no-op ``StorageHook``, blob storage being out of scope).
"""
from __future__ import annotations

from io import BytesIO

from fastapi import FastAPI, HTTPException, Request
from fastapi.exceptions import RequestValidationError
from PIL import Image, UnidentifiedImageError

from ..config import Config
from ..ingesting.core import StorageHook
from ..ingesting.utils import embed_locally, get_index
from ..ingesting.utils import get_feature_vector as _remote_feature_vector
from ..multipart import parse_form
from .utils import search

app = FastAPI(title="Image Retriever Service")
get_feature_vector = embed_locally if Config.EMBED_IN_PROCESS else _remote_feature_vector
storage = StorageHook()


def index():
    return get_index(Config.INDEX_NAME)


def _feature_fn(request: Request):
    """The app serving this request may embed its own way (service.py's one-process app sets
    ``app.state.feature_vector``); otherwise this module's ``get_feature_vector`` (the name the
    reference's tests monkeypatch)."""
    fn = getattr(request.app.state, "feature_vector", None)
    return fn if fn is not None else get_feature_vector


@app.get("/")
def read_root():
    return {"message": "Welcome to the Image Retriever API. Visit /docs to test."}


@app.get("/healthz")
def health_check():
    return {"status": "OK!"}


@app.post("/search_image")
async def search_image(request: Request):
    form = parse_form(await request.body(), request.headers.get("content-type", ""))
    f = form.get("file")
    if f is None:
        raise RequestValidationError([{"type": "missing", "loc": ("body", "file"), "msg": "Field required",
                                       "input": None}])
    feature_fn = _feature_fn(request)
    if not getattr(feature_fn, "validates_image", False):
        try:
            Image.open(BytesIO(f.data)).convert("RGB")
        except UnidentifiedImageError:
            raise HTTPException(status_code=400, detail="Uploaded file is not a valid image.")
    # else: the in-process embed validates the upload itself, with this route's 400 body, before
    # the model runs — a GPU-decodable JPEG is decoded once (on the GPU) instead of twice
    feature = feature_fn(f.data)
    ix = index()
    match_ids = search(ix, feature, top_k=Config.TOP_K)
    if not match_ids:
        return []
    response = ix.fetch(ids=match_ids)
    images_url = []
    for match_id in match_ids:
        if len(images_url) == Config.TOP_K:
            break
        vec = response.get("vectors", {}).get(match_id)
        if vec is None:
            continue
        gcs_path = vec.get("metadata", {}).get("gcs_path", "")
        images_url.append(storage.signed_url(gcs_path, None))
    return images_url
