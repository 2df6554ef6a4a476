"""Ingest service on the MI355X core (mirror of reference ``ingesting/main.py``).

Contract kept (``ingesting/main.py:91-168``):
  GET  /             → {"message": "Welcome to the Image Ingestion API. Visit /docs to test."}
  GET  /healthz      → {"status": "healthy"}
  POST /push_image   multipart ``file`` → {"message", "file_id", "gcs_path", "signed_url"}
                     400 "Only .jpg/.jpeg/.png allowed" / "Invalid image file"; 422 without ``file``
  POST /push_images  (batched form) repeated ``files`` → one such dict per image (ingesting.core.ingest_many)

``get_feature_vector`` is a module-level name, as in the reference (whose tests
monkeypatch ``ingesting.main.get_feature_vector``); by default it embeds in
process on the GPU (``RC_EMBED_IN_PROCESS=0`` POSTs to the /embed service like the
reference).  The index is opened on first use (the reference opens Pinecone at
import, ``:37``).  GCS is a no-op ``StorageHook`` (blob storage is out of scope);
OTel/Prometheus instrumentation is out of scope.
"""
from __future__ import annotations

from fastapi import FastAPI, Request
from fastapi.exceptions import RequestValidationError

from ..config import Config
from ..multipart import parse_form, parse_form_all
from . import core
from .utils import embed_locally, get_index
from .utils import get_feature_vector as _remote_feature_vector

app = FastAPI(title="Image Ingestion Service")
get_feature_vector = embed_locally if Config.EMBED_IN_PROCESS else _remote_feature_vector
storage = core.StorageHook()


def index():
    return get_index(Config.INDEX_NAME)


def _feature_fn(request: Request):
    """The app serving this request may embed its own way (service.py's one-process app sets
    ``app.state.feature_vector``); otherwise this module's ``get_feature_vector`` (the name the
    reference's tests monkeypatch)."""
    fn = getattr(request.app.state, "feature_vector", None)
    return fn if fn is not None else get_feature_vector


def _missing_file(field: str):
    return RequestValidationError([{"type": "missing", "loc": ("body", field), "msg": "Field required", "input": None}])


@app.get("/")
def read_root():
    return {"message": "Welcome to the Image Ingestion API. Visit /docs to test."}


@app.get("/healthz")
def health_check():
    return {"status": "healthy"}


@app.post("/push_image")
async def push_image(request: Request):
    form = parse_form(await request.body(), request.headers.get("content-type", ""))
    f = form.get("file")
    if f is None:
        raise _missing_file("file")
    return core.push_one(f.filename, f.data, index, content_type=f.content_type, storage=storage,
                         feature_fn=_feature_fn(request))


@app.post("/push_images")
async def push_images(request: Request):
    parts = parse_form_all(await request.body(), request.headers.get("content-type", "")).get("files")
    if not parts:
        raise _missing_file("files")
    return core.ingest_many([(f.filename, f.data, f.content_type) for f in parts], index, storage=storage)
