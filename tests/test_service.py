"""The one-process service (``…_amd/service.py``): every route of the reference's three pods
over one in-HBM index.

Reference deployment: ingest (``ingesting/main.py:37,172``) and retriever
(``retriever/main.py:36,173``) are two processes that open the SAME Pinecone index by
name.  The in-HBM index is process-local, so the drop-in serves both from one app; the
GPU test pushes through it and then searches through it.  ``/embed`` is also pinned by
value: the service loaded from a seed-1907 safetensors checkpoint returns the golden
vector (reference ``tests/test_embedding.py:32-38`` checks only the length).
"""
import io
import os

import numpy as np
import pytest
from fastapi.testclient import TestClient

from conftest import GOLDEN, import_pkg


@pytest.fixture(scope="module")
def svc():
    return TestClient(import_pkg("service").app)


@pytest.fixture(scope="module")
def fixture_jpeg():
    with open(os.path.join(GOLDEN, "test_image.jpeg"), "rb") as f:
        return f.read()


def test_service_serves_every_route(svc):
    paths = {getattr(r, "path", None) for r in import_pkg("service").app.router.routes}
    for p in ("/", "/healthz", "/embed", "/embed_batch", "/push_image", "/push_images", "/search_image"):
        assert p in paths, p
    assert svc.get("/healthz").json() == {"status": "healthy"}
    # the retriever pod answered {"status": "OK!"} (retriever/main.py:99-101): served on its own path
    assert svc.get("/healthz/retriever").json() == {"status": "OK!"}
    assert svc.get("/").json() == {"message": "Welcome to the Image Retrieval API. Visit /docs to test."}


def test_service_validation_contract(svc):
    """The per-route 400 / 422 responses of the three reference services (GPU-free)."""
    assert svc.post("/embed").status_code == 422
    assert svc.post("/push_image").status_code == 422
    assert svc.post("/search_image").status_code == 422
    bad = ("a.jpg", b"This is not an image.", "image/jpeg")
    r = svc.post("/embed", files={"file": bad})
    assert r.status_code == 400 and r.json()["detail"] == "Uploaded file is not a valid image."
    r = svc.post("/push_image", files={"file": bad})
    assert r.status_code == 400 and r.json()["detail"] == "Invalid image file"
    r = svc.post("/push_image", files={"file": ("a.gif", b"GIF89a", "image/gif")})
    assert r.status_code == 400 and r.json()["detail"] == "Only .jpg/.jpeg/.png allowed"
    r = svc.post("/search_image", files={"file": bad})
    assert r.status_code == 400 and r.json()["detail"] == "Uploaded file is not a valid image."


def test_service_embeds_in_process():
    """The one-process app embeds in process through its own app state; importing it rebinds
    nothing in the per-service modules (the name the reference's tests monkeypatch stays theirs)."""
    s = import_pkg("service")
    utils = import_pkg("ingesting.utils")
    assert s.app.state.feature_vector is utils.embed_locally
    for mod in ("ingesting.main", "retriever.main"):
        m = import_pkg(mod)
        assert getattr(m.app.state, "feature_vector", None) is None
        cfg = import_pkg("config").Config
        want = utils.embed_locally if cfg.EMBED_IN_PROCESS else utils.get_feature_vector
        assert m.get_feature_vector is want
    assert s.index is not None


def test_service_feature_vector_scoped_to_its_app(monkeypatch):
    """A monkeypatched retriever.main.get_feature_vector (reference tests/test_retriever.py:11-16)
    is what the retriever app uses; the one-process app keeps its own in-process embedder."""
    from starlette.requests import Request

    s = import_pkg("service")
    rm = import_pkg("retriever.main")
    fake = lambda _: [0.1] * 768  # noqa: E731
    monkeypatch.setattr(rm, "get_feature_vector", fake)
    req = lambda app: Request({"type": "http", "app": app, "headers": []})  # noqa: E731
    assert rm._feature_fn(req(rm.app)) is fake
    assert rm._feature_fn(req(s.app)) is import_pkg("ingesting.utils").embed_locally


def _jpeg(seed, w=224, h=224):
    from PIL import Image

    arr = np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)
    b = io.BytesIO()
    Image.fromarray(arr).save(b, format="JPEG", quality=85)
    return b.getvalue()


@pytest.mark.gpu
def test_service_push_then_search_one_index(svc, fixture_jpeg, cuda, monkeypatch):
    """push through the service, search through the service: the pushed image's URL is first,
    and both routes saw the one index."""
    cfg = import_pkg("config").Config
    monkeypatch.setattr(cfg, "INDEX_NAME", "one-process-service")
    r = svc.post("/push_image", files={"file": ("fixture.jpeg", fixture_jpeg, "image/jpeg")})
    assert r.status_code == 200
    first = r.json()
    others = [("files", (f"o{i}.jpg", _jpeg(100 + i, 300 - 8 * i, 168 + 4 * i), "image/jpeg")) for i in range(7)]
    r = svc.post("/push_images", files=others)
    assert r.status_code == 200 and len(r.json()) == 7
    batch = r.json()
    ix = import_pkg("service").index()
    assert len(ix) == 8
    r = svc.post("/search_image", files={"file": ("q.jpeg", fixture_jpeg, "image/jpeg")})
    assert r.status_code == 200
    urls = r.json()
    assert len(urls) == cfg.TOP_K
    assert urls[0] == first["signed_url"] and urls[0].endswith(first["gcs_path"])
    # an image of the batched push also finds itself first
    r = svc.post("/search_image", files={"file": others[3][1]})
    assert r.status_code == 200 and r.json()[0] == batch[3]["signed_url"]
    ix.close()
    import_pkg("ingesting.utils")._indexes.pop("one-process-service", None)


@pytest.mark.gpu
def test_embed_route_by_value_seed1907_checkpoint(svc, fixture_jpeg, cuda, tmp_path, monkeypatch):
    """POST /embed on the reference's fixture with the service loaded from a seed-1907
    safetensors checkpoint is within 1e-3 cosine of the transformers golden (fp32 tier)."""
    from safetensors.numpy import save_file

    from oracle.weights import seeded_vit_msn_weights

    save_file({k: np.ascontiguousarray(v) for k, v in seeded_vit_msn_weights(1907).items()},
              str(tmp_path / "model.safetensors"))
    emb = import_pkg("embedding.main")
    monkeypatch.setattr(emb.Config, "MODEL_PATH", str(tmp_path))
    emb.reset_embedder()
    try:
        r = svc.post("/embed", files={"file": ("test_image.jpeg", fixture_jpeg, "image/jpeg")})
        assert r.status_code == 200
        got = np.asarray(r.json(), dtype=np.float64)
        ref = np.load(os.path.join(GOLDEN, "test_image_embedding_seed1907.npy")).astype(np.float64).reshape(-1)
        cos = got @ ref / (np.linalg.norm(got) * np.linalg.norm(ref))
        assert got.shape == (768,) and 1.0 - cos < 1e-3, 1.0 - cos
    finally:
        emb.reset_embedder()


@pytest.mark.gpu
def test_search_image_truncated_jpeg_is_a_500(fixture_jpeg, cuda, monkeypatch):
    """/search_image no longer decodes the upload on the host before the in-process embed (which
    validates it itself): a truncated baseline JPEG passes the GPU decoder's header probe, the GPU
    decoder rejects the damaged scan, PIL decides — and PIL's OSError propagates as a 500, as the
    reference's validation decode (retriever/main.py:111-117) lets it; a non-image stays a 400."""
    cfg = import_pkg("config").Config
    monkeypatch.setattr(cfg, "INDEX_NAME", "truncated-jpeg-search")
    jpeg = import_pkg("jpeg")
    bad = fixture_jpeg[: len(fixture_jpeg) // 2]
    assert jpeg.is_gpu_decodable(bad)
    client = TestClient(import_pkg("service").app, raise_server_exceptions=False)
    r = client.post("/search_image", files={"file": ("t.jpeg", bad, "image/jpeg")})
    assert r.status_code == 500
    r = client.post("/search_image", files={"file": ("a.jpg", b"This is not an image.", "image/jpeg")})
    assert r.status_code == 400 and r.json()["detail"] == "Uploaded file is not a valid image."
    import_pkg("ingesting.utils")._indexes.pop("truncated-jpeg-search", None)
