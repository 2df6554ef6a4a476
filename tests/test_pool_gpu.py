"""Data-parallel embedding behind the product API (image embedding is plain data
parallel, no collectives; the reference scales its embedding pod by replicas,
``helm_charts/embedding/values.yaml:1``, and ingests one image per request,
``ingesting/main.py:124,156-158``).

``EmbedderPool`` = one ``rc_model`` per device.  On this 1-GPU pool its members share
cuda:0 (devices ``[0, 0]``): every code path of the multi-GPU pool runs (batch split,
concurrent rc_embed calls, per-member slices routed to their shards) and the results
must equal the single embedder's BIT FOR BIT (an image's arithmetic does not depend on
its batch).
"""
import io
import itertools

import numpy as np
import pytest

from conftest import import_pkg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def vitmod(cuda):
    return import_pkg("vit")


@pytest.fixture(scope="module")
def sd2():
    from oracle.weights import seeded_vit_msn_weights

    return seeded_vit_msn_weights(1907, num_layers=2)


def _images(n, seed):
    rng = np.random.default_rng(seed)
    sizes = ((224, 224), (168, 300), (224, 224), (97, 120))
    return [rng.integers(0, 256, sizes[i % len(sizes)] + (3,), dtype=np.uint8) for i in range(n)]


def test_pool_embed_equals_single_embedder(vitmod, sd2, cuda):
    import torch

    single = vitmod.VitMsnEmbedder(sd2, device=0, max_batch=16)
    pool = vitmod.EmbedderPool(sd2, [0, 0], max_batch=16)
    imgs = _images(37, 1)
    a, an = single.embed_images(imgs, normalized=True)
    b, bn = pool.embed_images(imgs, normalized=True)
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(an, bn)
    parts = pool.embed_parts(imgs, normalized=True, assign=pool.assign(37, base=5))
    assert sorted(p for pos, _, _ in parts for p in pos) == list(range(37))
    for mi, (pos, r, nr) in enumerate(parts):
        assert pos == [j for j in range(37) if (5 + j) % 2 == mi]  # round-robin from the base row
        assert torch.equal(r, a[pos]) and torch.equal(nr, an[pos])
    single.close()
    pool.close()


def test_pool_assign_follows_the_index_shards(vitmod, sd2, cuda):
    pool = vitmod.EmbedderPool(sd2, [0, 0], max_batch=4)
    # one member per shard on the same GPUs: image j (row base + j) -> member (base + j) % 2
    assert pool.assign(6, base=3, shard_devices=[0, 0]) == [1, 0, 1, 0, 1, 0]
    # a 4-shard index on this GPU: the members take turns per shard
    a = pool.assign(8, base=0, shard_devices=[0, 0, 0, 0])
    assert sorted(set(a)) == [0, 1]
    pool.close()


def _jpegs(n, seed):
    from PIL import Image

    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        w, h = ((224, 224), (300, 168))[i % 2]
        b = io.BytesIO()
        Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(b, format="JPEG", quality=85)
        out.append((f"p{i}.jpg", b.getvalue(), "image/jpeg"))
    return out


@pytest.fixture
def service_pool(cuda, monkeypatch):
    """The service singleton as a 2-member pool (RC_EMBED_DEVICES=0,0)."""
    emb = import_pkg("embedding.main")
    monkeypatch.setattr(emb.Config, "EMBED_DEVICES", "0,0")
    emb.reset_embedder()
    yield emb
    emb.reset_embedder()


def _ingest_reference(files_batches, cuda, monkeypatch):
    """What the single-GPU service stores for the same uploads (fresh singleton, one embedder)."""
    core = import_pkg("ingesting.core")
    index = import_pkg("index")
    emb = import_pkg("embedding.main")
    monkeypatch.setattr(emb.Config, "EMBED_DEVICES", "")
    emb.reset_embedder()
    ids = (f"q-{i}" for i in itertools.count())
    ix = index.Index("pool-ref", dimension=768, capacity=64, device=cuda, shards=2)
    resp = [core.ingest_many(b, ix, id_factory=lambda: next(ids)) for b in files_batches]
    emb.reset_embedder()
    return ix, resp


def test_pool_ingest_many_and_stream_equal_single(service_pool, cuda, monkeypatch):
    """ingest_many / ingest_stream through the pool: same responses, same stored vectors bit for
    bit, same search results as the single embedder; each image's vector went to the shard its
    row lives on from the member that embedded it (parts path of Index.upsert_tensor)."""
    import torch

    core = import_pkg("ingesting.core")
    index = import_pkg("index")
    ret = import_pkg("retriever.utils")
    from_vit = import_pkg("vit")
    files = _jpegs(30, 3)
    batches = [files[:11], files[11:30]]
    pool = service_pool.get_embedder()
    assert isinstance(pool, from_vit.EmbedderPool) and pool.devices == [0, 0]
    ids = (f"q-{i}" for i in itertools.count())
    ix = index.Index("pool-stream", dimension=768, capacity=64, device=cuda, shards=2)
    got = list(core.ingest_stream(iter(batches), ix, id_factory=lambda: next(ids)))
    ref_ix, want = _ingest_reference(batches, cuda, monkeypatch)
    assert got == want
    all_ids = [r["file_id"] for rs in got for r in rs]
    fa, fb = ix.fetch(all_ids), ref_ix.fetch(all_ids)
    for i in all_ids:
        assert fa["vectors"][i]["values"] == fb["vectors"][i]["values"]
        assert fa["vectors"][i]["metadata"] == fb["vectors"][i]["metadata"]
    sa, ra = ix.shard_set.search(torch.tensor([fa["vectors"]["q-4"]["values"]]), 10, len(ix))
    sb, rb = ref_ix.shard_set.search(torch.tensor([fb["vectors"]["q-4"]["values"]]), 10, len(ref_ix))
    assert torch.equal(sa, sb) and torch.equal(ra, rb)
    assert ret.search(ix, fa["vectors"]["q-7"]["values"], top_k=5)[0] == "q-7"
    ix.close()
    ref_ix.close()


def test_index_parts_upsert_equals_tensor_upsert(cuda):
    """Index.upsert_tensor with per-device parts (positions in any order, a repeated id across
    parts) stores what the single-tensor call stores."""
    import torch

    index = import_pkg("index")
    g = torch.Generator(device=cuda).manual_seed(3)
    v = torch.randn((9, 768), device=cuda, generator=g)
    ids = [f"x{i}" for i in range(8)] + ["x2"]  # x2 repeated: the last occurrence (position 8) wins
    a = index.Index("parts-a", dimension=768, capacity=16, device=cuda, shards=3)
    b = index.Index("parts-b", dimension=768, capacity=16, device=cuda, shards=3)
    a.upsert_tensor(ids, v)
    p0, p1 = [8, 0, 3, 6], [1, 2, 4, 5, 7]
    b.upsert_tensor(ids, [(p0, v[p0]), (p1, v[p1])])
    assert len(a) == len(b) == 8
    fa, fb = a.fetch(ids[:8]), b.fetch(ids[:8])
    for i in ids[:8]:
        assert fa["vectors"][i]["values"] == fb["vectors"][i]["values"]
    with pytest.raises(ValueError):
        b.upsert_tensor(ids, [(p0, v[p0])])  # positions not covered
    a.close()
    b.close()


def test_pool_decodes_per_member(vitmod, sd2, cuda):
    """decode_jpeg_for_embed on a pool: each member decodes its share with its own decoder (not
    everything through member 0), the images are bit-identical to one decoder's, and embedding
    them where they were decoded equals the single embedder."""
    import torch

    pool = vitmod.EmbedderPool(sd2, [0, 0], max_batch=4)
    single = vitmod.VitMsnEmbedder(sd2, device=0, max_batch=4)
    datas = [d for _, d, _ in _jpegs(9, 11)]
    ims = pool.decode_jpeg_for_embed(datas)
    assert all(m._jpeg is not None for m in pool.members)  # both members decoded
    ref = single.decode_jpeg_for_embed(datas)
    assert len(ims) == 9 and all(torch.equal(a, b) for a, b in zip(ims, ref.unbind(0)))
    raw, _ = pool.embed_images(ims, assign=pool.assign_by_location(ims))
    want, _ = single.embed_images(list(ref.unbind(0)))
    assert torch.equal(raw, want)
    assert pool.embed_jpeg(datas) == single.embed_jpeg(datas)
    pool.close()
    single.close()


def test_pool_concurrent_ingests_store_their_own_vectors(service_pool, cuda):
    """Two ingest_many calls racing on one pool and one index (the row plan is made
    outside the index lock): every id ends up with exactly the vector of its own image."""
    import concurrent.futures as cf

    core = import_pkg("ingesting.core")
    index = import_pkg("index")
    emb = service_pool
    a, b = _jpegs(12, 21), _jpegs(12, 22)
    ix = index.Index("pool-race", dimension=768, capacity=64, device=cuda, shards=2)
    with cf.ThreadPoolExecutor(2) as ex:
        fa = ex.submit(core.ingest_many, a, ix, None, (lambda c=itertools.count(): f"a-{next(c)}"))
        fb = ex.submit(core.ingest_many, b, ix, None, (lambda c=itertools.count(): f"b-{next(c)}"))
        ra, rb = fa.result(), fb.result()
    assert len(ix) == 24
    for files, resp in ((a, ra), (b, rb)):
        want = emb.embed_many([f[1] for f in files])
        got = ix.fetch([r["file_id"] for r in resp])["vectors"]
        for r, w in zip(resp, want):
            assert np.allclose(got[r["file_id"]]["values"], w, rtol=1e-5, atol=1e-6)
    assert ix.shard_set.cross_device_rows == 0  # one GPU: nothing crossed
    ix.close()
