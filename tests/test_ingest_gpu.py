"""Ingest → retrieve through the reference API, on the GPU.

* The batched ingest core (``ingesting.core.ingest_many``)
  returns, per image, what a loop of single ``/push_image`` calls returns
  (reference ``ingesting/main.py:101-168``), and the index it fills answers
  ``search`` (``retriever/utils.py:59-66``) like the single-push index.
* ``ingest_stream`` (bulk ingest: decode of batch i+1 under the embed of batch i)
  returns per batch what ``ingest_many`` returns and stores the same bits.
* The ``/push_image`` → ``/search_image`` services (reference
  ``tests/test_ingesting.py:47-50``, ``tests/test_retriever.py:46-54``).
* BASELINE config 5, single-GPU shape: 65,536 synthetic images embedded on the
  device and upserted (device-resident vectors, string ids) into a round-robin
  sharded fp16 index, then 1024 queries top-100: MFMA path == exact scan bit for
  bit, every query finds its own image first, and the float64 oracle agrees on
  a query sample.
"""
import io
import itertools

import numpy as np
import pytest

from conftest import import_pkg
from oracle.cosine_topk import cosine_topk, topk_equal_modulo_ties

pytestmark = pytest.mark.gpu


def _jpegs(n, seed, sizes=((224, 224), (300, 168), (64, 80))):
    from PIL import Image

    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        w, h = sizes[i % len(sizes)]
        arr = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        b = io.BytesIO()
        if i % 7 == 3:
            Image.fromarray(arr).save(b, format="PNG")
            out.append((f"img{i}.png", b.getvalue(), "image/png"))
        else:
            Image.fromarray(arr).save(b, format="JPEG", quality=85)
            out.append((f"img{i}.JPG", b.getvalue(), "image/jpeg"))
    return out


def test_ingest_many_equals_single_pushes(cuda):
    core = import_pkg("ingesting.core")
    index = import_pkg("index")
    emb = import_pkg("embedding.main")
    files = _jpegs(40, 1)
    ids_a = (f"id-{i}" for i in itertools.count())
    ids_b = (f"id-{i}" for i in itertools.count())
    batch_ix = index.Index("batch", dimension=768, capacity=16, device=cuda, shards=2)
    single_ix = index.Index("single", dimension=768, capacity=16, device=cuda)
    got = core.ingest_many(files, batch_ix, id_factory=lambda: next(ids_a))
    want = [core.push_one(f[0], f[1], single_ix, content_type=f[2], feature_fn=emb.embed_bytes,
                          id_factory=lambda: next(ids_b)) for f in files]
    assert got == want
    assert got[3]["gcs_path"] == "images/id-3.png" and got[0]["gcs_path"] == "images/id-0.jpg"
    assert all(set(r) == {"message", "file_id", "gcs_path", "signed_url"} for r in got)
    assert all(r["signed_url"].startswith("https://") for r in got)
    # the same vectors went in: fetch and search agree between the two indexes
    ids = [r["file_id"] for r in got]
    fa, fb = batch_ix.fetch(ids), single_ix.fetch(ids)
    for i in ids:
        assert np.array_equal(fa["vectors"][i]["values"], fb["vectors"][i]["values"])
        assert fa["vectors"][i]["metadata"] == fb["vectors"][i]["metadata"]
    ret = import_pkg("retriever.utils")
    q = emb.embed_bytes(files[5][1])
    assert ret.search(batch_ix, q, top_k=5) == ret.search(single_ix, q, top_k=5)
    assert ret.search(batch_ix, q, top_k=5)[0] == "id-5"
    batch_ix.close()
    single_ix.close()


def test_ingest_stream_equals_ingest_many_per_batch(cuda):
    """The pipelined bulk ingest (decode of batch i+1 under the embed of batch i) returns, batch
    by batch, what ingest_many returns, and stores the same vectors bit for bit."""
    core = import_pkg("ingesting.core")
    index = import_pkg("index")
    files = _jpegs(48, 5)  # JPEG + PNG, three sizes
    batches = [files[:16], files[16:40], files[40:]]
    ids_a = (f"s-{i}" for i in itertools.count())
    ids_b = (f"s-{i}" for i in itertools.count())
    ix_s = index.Index("stream", dimension=768, capacity=64, device=cuda, shards=2)
    ix_m = index.Index("many", dimension=768, capacity=64, device=cuda)
    got = list(core.ingest_stream(iter(batches), ix_s, id_factory=lambda: next(ids_a)))
    want = [core.ingest_many(b, ix_m, id_factory=lambda: next(ids_b)) for b in batches]
    assert got == want and [len(r) for r in got] == [16, 24, 8]
    ids = [r["file_id"] for rs in got for r in rs]
    fa, fb = ix_s.fetch(ids), ix_m.fetch(ids)
    for i in ids:
        assert np.array_equal(fa["vectors"][i]["values"], fb["vectors"][i]["values"])
        assert fa["vectors"][i]["metadata"] == fb["vectors"][i]["metadata"]
    ix_s.close()
    ix_m.close()


def test_ingest_stream_stops_at_an_invalid_batch(cuda):
    from fastapi import HTTPException

    core = import_pkg("ingesting.core")
    index = import_pkg("index")
    ix = index.Index("stream-rej", dimension=768, capacity=32, device=cuda)
    good = _jpegs(6, 7)
    bad = _jpegs(2, 8) + [("bad.jpg", b"This is not an image.", "image/jpeg")]
    gen = core.ingest_stream(iter([good, bad, _jpegs(4, 9)]), ix)
    assert len(next(gen)) == 6
    with pytest.raises(HTTPException) as e:
        next(gen)
    assert e.value.status_code == 400 and e.value.detail == "Invalid image file"
    assert len(ix) == 6  # the invalid batch and the ones after it are not ingested
    ix.close()


def test_ingest_many_rejects_before_ingesting(cuda):
    from fastapi import HTTPException

    core = import_pkg("ingesting.core")
    index = import_pkg("index")
    ix = index.Index("rej", dimension=768, capacity=8, device=cuda)
    files = _jpegs(3, 2) + [("bad.jpg", b"This is not an image.", "image/jpeg")]
    with pytest.raises(HTTPException) as e:
        core.ingest_many(files, ix)
    assert e.value.status_code == 400 and e.value.detail == "Invalid image file"
    assert len(ix) == 0
    ix.close()


def test_push_then_search_services(cuda, monkeypatch):
    from fastapi.testclient import TestClient

    cfg = import_pkg("config").Config
    monkeypatch.setattr(cfg, "INDEX_NAME", "service-test")
    ing = TestClient(import_pkg("ingesting.main").app)
    ret = TestClient(import_pkg("retriever.main").app)
    files = _jpegs(6, 3)
    r = ing.post("/push_image", files={"file": files[0][:2] + (files[0][2],)})
    assert r.status_code == 200 and set(r.json()) == {"message", "file_id", "gcs_path", "signed_url"}
    first = r.json()
    r = ing.post("/push_images", files=[("files", f) for f in files[1:]])
    assert r.status_code == 200 and len(r.json()) == 5
    r = ret.post("/search_image", files={"file": files[0][:2] + (files[0][2],)})
    assert r.status_code == 200
    urls = r.json()
    assert 0 < len(urls) <= cfg.TOP_K and all(u.startswith("https://") for u in urls)
    assert urls[0].endswith(first["gcs_path"])


def test_config5_ingest_then_retrieve_single_gpu(cuda):
    import torch

    index = import_pkg("index")
    vit = import_pkg("vit")
    n, B, nq, k = 65_536, 256, 1024, 100
    model = vit.VitMsnEmbedder(vit.random_state_dict(seed=0), device=0, max_batch=B)
    ix = index.Index("config5", dimension=768, dtype="float16", capacity=n, device=cuda, shards=2)
    g = torch.Generator(device="cuda").manual_seed(6000)
    qpick = torch.arange(0, n, n // nq)[:nq]  # image ids used as queries
    queries = torch.empty((nq, 768), device="cuda")
    for b0 in range(0, n, B):
        imgs = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device="cuda", generator=g)
        raw, _ = model.embed(imgs, normalized=False)
        ix.upsert_tensor([f"img-{i}" for i in range(b0, b0 + B)], raw)
        sel = (qpick >= b0) & (qpick < b0 + B)
        if sel.any():
            queries[sel.nonzero().reshape(-1).cuda()] = raw[(qpick[sel] - b0).cuda()]
    assert len(ix) == n
    ss = ix.shard_set
    s, r = ss.search(queries, k, n, mode="mfma")
    assert (r[:, 0].cpu() == qpick).all(), "every query image must find itself first"
    assert (s[:, :-1] >= s[:, 1:]).all()
    samp = torch.arange(0, nq, 16)
    s2, r2 = ss.search(queries[samp.cuda()], k, n, mode="scan")
    assert torch.equal(r[samp.cuda()], r2) and torch.equal(s[samp.cuda()], s2)
    stored = ss.fetch_rows(np.arange(n), stored=True).numpy()
    qn = queries[samp[:16].cuda()].cpu().numpy()
    ref_r, ref_s = cosine_topk(stored, qn, k, rows_normalized=True)
    for j in range(16):
        assert topk_equal_modulo_ties(r2[j].cpu().numpy(), s2[j].cpu().numpy(), ref_r[j], ref_s[j])
    res = ix.query_batch(queries[:8], top_k=5)
    assert [m["matches"][0]["id"] for m in res] == [f"img-{int(i)}" for i in qpick[:8]]
    model.close()
    ix.close()
