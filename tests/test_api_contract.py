"""HTTP / helper contract of the reference's API surface (mirrors reference tests/test_*.py).

Reference pins (tests/test_embedding.py:26-50, tests/test_ingesting.py, tests/test_retriever.py):
healthz bodies, 400 detail string on a non-image, 422 on a missing file, /embed →
flat list of floats; search → ids best first, ValueError on an empty embedding;
get_feature_vector → HTTPException(500) on any failure.  CPU tests exercise only
paths that need no GPU; the valid-image embed runs under -m gpu.
"""
import os

import pytest
from fastapi import HTTPException
from fastapi.testclient import TestClient

from conftest import GOLDEN, import_pkg


@pytest.fixture(scope="module")
def client():
    return TestClient(import_pkg("embedding.main").app)


@pytest.fixture(scope="session")
def test_image_bytes():
    with open(os.path.join(GOLDEN, "test_image.jpeg"), "rb") as f:
        return f.read()


def test_embedding_health(client):
    r = client.get("/healthz")
    assert r.status_code == 200 and r.json()["status"] == "healthy"


def test_embedding_root(client):
    assert client.get("/").json() == {"message": "Welcome to ViT-MSN Embedding API. Visit /docs to test."}


def test_embed_invalid_image_type(client):
    files = {"file": ("fake.txt", b"This is not an image at all.", "text/plain")}
    r = client.post("/embed", files=files)
    assert r.status_code == 400
    assert r.json()["detail"] == "Uploaded file is not a valid image."


def test_embed_no_file(client):
    assert client.post("/embed").status_code == 422


def test_embed_wrong_field_name(client, test_image_bytes):
    r = client.post("/embed", files={"image": ("a.jpeg", test_image_bytes, "image/jpeg")})
    assert r.status_code == 422
    assert r.json()["detail"][0]["loc"] == ["body", "file"]


def test_multipart_parser_roundtrip(test_image_bytes):
    mp = import_pkg("multipart")
    import httpx

    req = httpx.Request("POST", "http://x/embed", files={"file": ("t.jpeg", test_image_bytes, "image/jpeg")})
    body = req.read()
    form = mp.parse_form(body, req.headers["content-type"])
    assert form["file"].data == test_image_bytes
    assert form["file"].filename == "t.jpeg"


def test_search_empty_embedding_raises():
    utils = import_pkg("retriever.utils")
    with pytest.raises(ValueError, match="Input embedding is empty"):
        utils.search(None, [], 5)


def test_search_returns_ids_best_first():
    utils = import_pkg("retriever.utils")

    class FakeIndex:
        def query(self, vector, top_k, include_values):
            assert include_values is True and top_k == 5
            return {"matches": [{"id": "b", "score": 0.9}, {"id": "a", "score": 0.5}]}

    assert utils.search(FakeIndex(), [0.1] * 768, 5) == ["b", "a"]


def test_get_feature_vector_posts_file(monkeypatch, test_image_bytes):
    utils = import_pkg("ingesting.utils")
    seen = {}

    class Resp:
        def raise_for_status(self):
            pass

        def json(self):
            return [0.1] * 768

    def fake_post(url, files):
        seen["url"], seen["files"] = url, files
        return Resp()

    monkeypatch.setattr(utils.requests, "post", fake_post)
    assert utils.get_feature_vector(test_image_bytes) == [0.1] * 768
    assert seen["files"]["file"] == ("image.jpg", test_image_bytes, "image/jpeg")
    assert seen["url"] == import_pkg("config").Config.EMBEDDING_SERVICE_URL


def test_get_feature_vector_failure_is_500(monkeypatch):
    utils = import_pkg("ingesting.utils")

    def boom(url, files):
        raise ConnectionError("down")

    monkeypatch.setattr(utils.requests, "post", boom)
    with pytest.raises(HTTPException) as e:
        utils.get_feature_vector(b"x")
    assert e.value.status_code == 500
    assert e.value.detail == "Failed to get feature vector from embedding service"


def test_config_names_match_reference():
    C = import_pkg("config").Config
    assert C.INPUT_RESOLUTION == 768 and C.TOP_K == 5 and C.INDEX_NAME == "mlops1-project"


@pytest.mark.gpu
def test_embed_valid_image(client, test_image_bytes, cuda):
    files = {"file": ("test_image.jpeg", test_image_bytes, "image/jpeg")}
    r = client.post("/embed", files=files)
    assert r.status_code == 200
    vec = r.json()
    assert isinstance(vec, list) and len(vec) == 768 and all(isinstance(v, float) for v in vec)


@pytest.mark.gpu
def test_embed_batch_matches_single(client, test_image_bytes, cuda):
    files = [("files", ("a.jpeg", test_image_bytes, "image/jpeg")), ("files", ("b.jpeg", test_image_bytes, "image/jpeg"))]
    r = client.post("/embed_batch", files=files)
    assert r.status_code == 200
    vs = r.json()
    single = client.post("/embed", files={"file": ("t.jpeg", test_image_bytes, "image/jpeg")}).json()
    assert len(vs) == 2 and vs[0] == single and vs[1] == single


@pytest.mark.gpu
def test_ingest_then_retrieve_end_to_end(test_image_bytes, cuda):
    """push_image's upsert (ingesting/main.py:156-158) then search_image's query (retriever/main.py:128)."""
    ing = import_pkg("ingesting.utils")
    ret = import_pkg("retriever.utils")
    idx = ing.get_index("e2e-test", capacity=64)
    vec = ing.embed_locally(test_image_bytes)
    idx.upsert([("img-0", vec, {"gcs_path": "images/img-0.jpeg", "filename": "x.jpeg"})])
    import numpy as np

    rng = np.random.default_rng(0)
    idx.upsert([(f"noise-{i}", rng.standard_normal(768).tolist(), {}) for i in range(20)])
    ids = ret.search(idx, vec, top_k=5)
    assert ids[0] == "img-0" and len(ids) == 5
    got = idx.fetch(ids=ids[:1])["vectors"]["img-0"]
    assert got["metadata"]["gcs_path"] == "images/img-0.jpeg"
    assert np.allclose(got["values"], vec, rtol=1e-5, atol=1e-5)
    res = idx.query(vector=vec, top_k=3, include_metadata=True)
    assert res["matches"][0]["id"] == "img-0" and abs(res["matches"][0]["score"] - 1.0) < 1e-5
    idx.upsert([("img-0", (-np.asarray(vec)).tolist(), {})])  # overwrite by id
    assert ret.search(idx, vec, top_k=21)[-1] == "img-0"
    with pytest.raises(ValueError):
        idx.upsert([("bad", [0.0] * 768, {})])
    with pytest.raises(ValueError):
        idx.query(vector=[1.0] * 10, top_k=3)


@pytest.mark.gpu
def test_embed_gpu_jpeg_path_equals_pil_path(client, test_image_bytes, cuda, monkeypatch):
    """/embed on a baseline JPEG decodes on the GPU; the vector equals the host-PIL-decode path's."""
    import io

    import numpy as np
    from PIL import Image

    main = import_pkg("embedding.main")
    J = import_pkg("jpeg")
    assert J.is_gpu_decodable(test_image_bytes)
    gpu_vec = client.post("/embed", files={"file": ("t.jpeg", test_image_bytes, "image/jpeg")}).json()
    monkeypatch.setattr(main.Config, "GPU_JPEG", False)
    pil_vec = client.post("/embed", files={"file": ("t.jpeg", test_image_bytes, "image/jpeg")}).json()
    assert gpu_vec == pil_vec
    monkeypatch.setattr(main.Config, "GPU_JPEG", True)
    b = io.BytesIO()
    Image.fromarray(np.full((40, 30, 3), 90, np.uint8)).save(b, format="PNG")
    r = client.post("/embed_batch", files=[("files", ("a.png", b.getvalue(), "image/png")),
                                          ("files", ("b.jpeg", test_image_bytes, "image/jpeg"))])
    assert r.status_code == 200
    vs = r.json()
    assert len(vs) == 2 and vs[1] == gpu_vec and len(vs[0]) == 768


# ------------------------------------------------ ingest / retriever services --
# reference tests/test_ingesting.py:41-55 and tests/test_retriever.py:40-59 (the
# success paths need the GPU and run under -m gpu in test_ingest_gpu.py)
@pytest.fixture(scope="module")
def ingest_client():
    return TestClient(import_pkg("ingesting.main").app)


@pytest.fixture(scope="module")
def retriever_client():
    return TestClient(import_pkg("retriever.main").app)


def test_ingest_health_and_root(ingest_client):
    assert ingest_client.get("/healthz").json() == {"status": "healthy"}
    assert ingest_client.get("/").json() == {"message": "Welcome to the Image Ingestion API. Visit /docs to test."}


def test_batched_routes_share_the_single_route_contract(client, ingest_client):
    """/embed_batch and /push_images parse with the same parser as /embed and /push_image:
    422 without the field or without a multipart body, 400 with the reference's detail for
    a non-image (GPU-free: validation runs before the model)."""
    assert client.post("/embed_batch").status_code == 422
    assert client.post("/embed_batch", content=b"x", headers={"content-type": "text/plain"}).status_code == 422
    assert client.post("/embed_batch", files=[("file", ("a.jpg", b"x", "image/jpeg"))]).status_code == 422
    r = client.post("/embed_batch", files=[("files", ("a.txt", b"This is not an image at all.", "text/plain"))])
    assert r.status_code == 400 and r.json() == {"detail": "Uploaded file is not a valid image."}
    r = client.post("/embed", files={"file": ("a.txt", b"This is not an image at all.", "text/plain")})
    assert r.status_code == 400 and r.json() == {"detail": "Uploaded file is not a valid image."}
    assert ingest_client.post("/push_images", files=[("file", ("a.jpg", b"x", "image/jpeg"))]).status_code == 422
    r = ingest_client.post("/push_images", files=[("files", ("a.jpg", b"This is not an image.", "image/jpeg"))])
    assert r.status_code == 400 and r.json()["detail"] == "Invalid image file"


def test_parse_form_all_keeps_repeated_fields():
    mp = import_pkg("multipart")
    from urllib3 import encode_multipart_formdata

    body, ctype = encode_multipart_formdata([("files", ("a.jpg", b"A", "image/jpeg")), ("other", "x"),
                                             ("files", ("b.png", b"BB", "image/png"))])
    allf = mp.parse_form_all(body, ctype)
    assert [(f.filename, f.data, f.content_type) for f in allf["files"]] == [("a.jpg", b"A", "image/jpeg"),
                                                                             ("b.png", b"BB", "image/png")]
    assert mp.parse_form(body, ctype)["files"].data == b"BB"  # one part per field: the last, as form.get
    assert mp.parse_form_all(b"x", "text/plain") == {}


def test_push_no_file(ingest_client):
    assert ingest_client.post("/push_image").status_code == 422
    assert ingest_client.post("/push_images").status_code == 422


def test_push_bad_extension(ingest_client, test_image_bytes):
    r = ingest_client.post("/push_image", files={"file": ("a.gif", test_image_bytes, "image/gif")})
    assert r.status_code == 400 and r.json()["detail"] == "Only .jpg/.jpeg/.png allowed"
    r = ingest_client.post("/push_images", files=[("files", ("a.jpeg", test_image_bytes, "image/jpeg")),
                                                  ("files", ("b.txt", b"x", "text/plain"))])
    assert r.status_code == 400 and r.json()["detail"] == "Only .jpg/.jpeg/.png allowed"


def test_push_invalid_image(ingest_client):
    r = ingest_client.post("/push_image", files={"file": ("a.jpg", b"This is not an image.", "image/jpeg")})
    assert r.status_code == 400 and r.json()["detail"] == "Invalid image file"


def test_retriever_health_and_root(retriever_client):
    assert retriever_client.get("/healthz").json() == {"status": "OK!"}
    assert retriever_client.get("/").json() == {"message": "Welcome to the Image Retriever API. Visit /docs to test."}


def test_search_no_file_and_invalid(retriever_client):
    assert retriever_client.post("/search_image").status_code == 422
    r = retriever_client.post("/search_image", files={"file": ("a.jpg", b"This is not an image.", "image/jpeg")})
    assert r.status_code == 400 and r.json()["detail"] == "Uploaded file is not a valid image."


def test_index_devices_spec(monkeypatch):
    utils = import_pkg("ingesting.utils")
    assert utils.index_devices("0,2,4") == [0, 2, 4]
    assert utils.index_devices("", shards=3) == [None, None, None]


def test_query_vector_parsing_matches_numpy():
    """Index.query's request path turns the JSON list into f32 through array('f'); it must give
    numpy's f32 rounding bit for bit for floats, ints, numpy scalars and tuples, and keep the
    reference's errors (wrong dimension, all-zero vector) — no GPU needed."""
    import numpy as np
    import torch

    idx = import_pkg("index")
    rng = np.random.default_rng(5)
    vals = (rng.standard_normal(768) * 10.0 ** rng.integers(-8, 8, 768)).tolist()
    ref = np.asarray(vals, dtype=np.float32)
    for v in (vals, tuple(vals), [np.float64(x) for x in vals], np.asarray(vals), torch.tensor(vals, dtype=torch.float64)):
        got = idx._as_vector_np(v, 768)
        assert got.shape == (1, 768) and got.dtype == np.float32 and got.flags.c_contiguous
        assert np.array_equal(got[0], ref)
    ints = list(range(1, 769))
    assert np.array_equal(idx._as_vector_np(ints, 768)[0], np.arange(1, 769, dtype=np.float32))
    with pytest.raises(ValueError):
        idx._as_vector_np(vals[:10], 768)
    with pytest.raises(ValueError):
        idx._as_vector_np([0.0] * 768, 768)
    with pytest.raises((ValueError, TypeError)):
        idx._as_vector_np(["a"] * 768, 768)
