"""One GPU-owning process that serves the reference's three pods over ONE in-HBM index.

In the reference the ingest pod (``ingesting/main.py``, port 5001, ``:172``) and the
retriever pod (``retriever/main.py``, port 5002, ``:173``) are separate processes that
both open the same remote Pinecone index by name (``ingesting/main.py:37``,
``retriever/main.py:36``), and both call the embedding pod (``embedding/main.py``,
port 5000) over HTTP.  Here the index lives in the HBM of the process that created
it (``ingesting.utils.get_index`` keeps one ``Index`` per name per process), so two
separate ingest and retriever processes would each hold their own index and the
retriever's would stay empty.  The drop-in deployment therefore collapses the three
pods into this one app: every route of the three services, one embedder, and one
``get_index(Config.INDEX_NAME)`` that ``/push_image(s)`` write and ``/search_image``
reads.  The per-service apps stay importable for their own contract tests.

  GET  /              → {"message": "Welcome to the Image Retrieval API. Visit /docs to test."}
  GET  /healthz       → {"status": "healthy"}  (the embedding and ingest pods' body)
  GET  /healthz/retriever → {"status": "OK!"}  (the retriever pod's body, retriever/main.py:99-101,
                          for a probe or client of the old retriever URL that checks the body)
  POST /embed, /embed_batch                  (embedding/main.py:88-124)
  POST /push_image, /push_images             (ingesting/main.py:101-168)
  POST /search_image                         (retriever/main.py:104-169)

Run: ``uvicorn "<package>.service:app" --host 0.0.0.0 --port 5000`` (one process: the
index is process-local, so do not start several uvicorn workers).
"""
from __future__ import annotations

from fastapi import FastAPI
from fastapi.routing import APIRoute

from .config import Config
from .embedding import main as embedding_main
from .ingesting import main as ingesting_main
from .ingesting.utils import embed_locally, get_index
from .retriever import main as retriever_main

app = FastAPI(title="Image Retrieval Service (MI355X, one process)")

_OWN = {"/", "/healthz"}
SERVICE_APPS = (embedding_main.app, ingesting_main.app, retriever_main.app)


def _mount(sub: FastAPI) -> None:
    for route in sub.router.routes:
        if isinstance(route, APIRoute) and route.path not in _OWN:
            app.router.routes.append(route)


for _sub in SERVICE_APPS:
    _mount(_sub)

# /embed is served by this very process: the ingest and retrieve routes embed in process
# (an HTTP hop to ourselves would only add latency).  Scoped to this app: the mounted route
# handlers read request.app.state.feature_vector, so the per-service apps (and the
# module-level get_feature_vector the reference's tests monkeypatch) are left as they are.
app.state.feature_vector = embed_locally


def index():
    """The one index every route of this app reads and writes."""
    return get_index(Config.INDEX_NAME)


@app.get("/")
def read_root():
    return {"message": "Welcome to the Image Retrieval API. Visit /docs to test."}


@app.get("/healthz")
def health_check():
    return {"status": "healthy"}


@app.get("/healthz/retriever")
def health_check_retriever():
    return retriever_main.health_check()
