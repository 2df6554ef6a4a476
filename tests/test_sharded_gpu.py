"""Multi-shard index behind the reference API (get_index → upsert / query / fetch).

Reference: ``get_index`` (``ingesting/utils.py:23-38``), ``index.upsert``
(``ingesting/main.py:156-158``), ``search``/``index.query`` (``retriever/utils.py:
59-66``), ``index.fetch`` (``retriever/main.py:142``).  The property: an index
row-sharded round-robin over n shards (``rc_sharded``: per-shard searches, then
rc_topk_merge keyed by (score desc, global row asc)) returns EXACTLY what one
shard holding the same vectors returns — same ids, same scores, same tie order —
in every search mode, including shards that are still empty.  The one-GPU box
puts every shard on cuda:0; the routing, merge and per-shard streams are the
same code a multi-GPU placement runs (its peer copies aside).
"""
import os
import socket

import numpy as np
import pytest

from conftest import REPO, import_pkg
from oracle.cosine_topk import cosine_topk, topk_equal_modulo_ties

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def idxmod(cuda):
    return import_pkg("index")


def _items(rng, n, dim, prefix="v", start=0):
    X = rng.standard_normal((n, dim)).astype(np.float32)
    return X, [(f"{prefix}{start + i}", X[i].tolist(), {"gcs_path": f"images/{start + i}.jpg", "n": start + i})
               for i in range(n)]


@pytest.mark.parametrize("dtype,shards,remote", [("float32", 3, False), ("float16", 4, False), ("bfloat16", 2, False),
                                                 ("float16", 3, True), ("float32", 4, True)])
def test_sharded_index_equals_single_shard(idxmod, cuda, dtype, shards, remote, monkeypatch):
    """A multi-shard index answers exactly like one shard.  remote: every shard but the leader
    is driven through the cross-device path (rc_sharded_force_remote: subset gather on the
    leader, peer copies of queries / subsets / result lists, leader merge) — the code the
    8-GPU node runs, exercised on one GPU."""
    rng = np.random.default_rng(7)
    dim = 768
    one = idxmod.Index("one", dimension=dim, dtype=dtype, capacity=512, device=cuda)
    many = idxmod.Index("many", dimension=dim, dtype=dtype, capacity=512, device=cuda, shards=shards)
    if remote:
        many.shard_set.force_remote()
    X, items = _items(rng, 3000, dim)
    X[1001] = X[17]  # exact ties on different shards (17 % n != 1001 % n for n = 2, 3, 4)
    items[1001] = ("v1001", X[17].tolist(), items[1001][2])
    for ix in (one, many):  # three calls, capacity grows 512 -> 4096 on the way
        ix.upsert(items[:1000])
        ix.upsert(items[1000:2500])
        ix.upsert(items[2500:] + [("v5", X[9].tolist(), {"over": 1})])  # overwrite by id
    assert len(one) == len(many) == 3000 and many.capacity >= 3000
    assert many.describe_index_stats()["shards"] == shards
    Q = rng.standard_normal((70, dim)).astype(np.float32)
    Q[0] = X[17]
    for k in (1, 5, 100, 256):
        a = one.query(vector=Q[0].tolist(), top_k=k, include_metadata=True, include_values=True)
        b = many.query(vector=Q[0].tolist(), top_k=k, include_metadata=True, include_values=True)
        assert a == b
    assert [m["id"] for m in b["matches"][:2]] == ["v17", "v1001"]  # tie → lower row first
    for mode in ("scan", "auto") + (("mfma",) if dtype != "float32" else ()):
        ra = one.query_batch(Q, top_k=50, mode=mode)
        rb = many.query_batch(Q, top_k=50, mode=mode)
        assert ra == rb, mode
    ids = ["v0", "v5", "v2999", "missing", "v1001"]
    assert one.fetch(ids) == many.fetch(ids)
    assert many.fetch(["v5"])["vectors"]["v5"]["metadata"] == {"over": 1}
    one.close()
    many.close()


def test_sharded_matches_oracle(idxmod, cuda):
    rng = np.random.default_rng(3)
    many = idxmod.Index("o", dimension=512, dtype="float16", capacity=20_000, device=cuda, shards=5)
    X, items = _items(rng, 20_000, 512)
    many.upsert(items)
    Q = rng.standard_normal((12, 512)).astype(np.float32)
    stored = many.shard_set.fetch_rows(np.arange(20_000), stored=True).numpy()
    ref_r, ref_s = cosine_topk(stored, Q, 10, rows_normalized=True)
    res = many.query_batch(Q, top_k=10, mode="mfma")
    for q in range(12):
        got = res[q]["matches"]
        r = np.array([int(m["id"][1:]) for m in got])
        s = np.array([m["score"] for m in got], dtype=np.float32)
        assert topk_equal_modulo_ties(r, s, ref_r[q], ref_s[q])
    many.close()


def test_empty_and_partly_filled_shards(idxmod, cuda):
    """Rows route round-robin: with 2 vectors over 4 shards, shards 2 and 3 are empty and must
    answer (-inf, -1) lists in every mode instead of failing."""
    rng = np.random.default_rng(1)
    ix = idxmod.Index("e", dimension=512, dtype="float16", capacity=64, device=cuda, shards=4)
    assert ix.query(vector=rng.standard_normal(512).tolist(), top_k=5) == {"matches": [], "namespace": ""}
    X, items = _items(rng, 2, 512)
    ix.upsert(items)
    for mode in ("scan", "mfma", "auto"):
        res = ix.query_batch(np.concatenate([X, X]), top_k=5, mode=mode)
        assert [[m["id"] for m in r["matches"]] for r in res] == [["v0", "v1"], ["v1", "v0"]] * 2
    ss = ix.shard_set
    s, r = ss.search(__import__("torch").from_numpy(X), 5, 2, mode="mfma")
    assert (r[:, 2:] == -1).all() and s[:, 2:].isneginf().all()
    ix.close()


def test_upsert_repeated_id_in_one_call_keeps_last(idxmod, cuda):
    """a repeated id in one upsert call must not write one row slot twice."""
    rng = np.random.default_rng(2)
    ix = idxmod.Index("d", dimension=768, capacity=16, device=cuda, shards=2)
    X = rng.standard_normal((3, 768)).astype(np.float32)
    r = ix.upsert([("a", X[0].tolist()), ("b", X[1].tolist()), ("a", X[2].tolist(), {"last": True})])
    assert r == {"upserted_count": 2} and len(ix) == 2
    got = ix.fetch(["a"])["vectors"]["a"]
    assert np.allclose(got["values"], X[2], rtol=1e-6, atol=1e-6) and got["metadata"] == {"last": True}
    m = ix.query(vector=X[2].tolist(), top_k=1)["matches"][0]
    assert m["id"] == "a" and abs(m["score"] - 1.0) < 1e-6
    import torch

    ix.upsert_tensor(["c", "c"], torch.from_numpy(X[:2]).cuda())
    assert np.allclose(ix.fetch(["c"])["vectors"]["c"]["values"], X[1], atol=1e-6)
    ix.close()


def test_top_k_limits(idxmod, cuda):
    ix = idxmod.Index("t", dimension=64, capacity=8, device=cuda)
    ix.upsert([("a", [1.0] * 64)])
    with pytest.raises(ValueError):
        ix.query(vector=[1.0] * 64, top_k=257)  # no silent clamp
    with pytest.raises(ValueError):
        ix.query(vector=[1.0] * 64, top_k=0)
    assert len(ix.query(vector=[1.0] * 64, top_k=256)["matches"]) == 1
    ix.close()


def test_get_index_multi_shard(cuda, monkeypatch):
    """get_index (reference ingesting/utils.py:23-38) over RC_INDEX_SHARDS shards."""
    utils = import_pkg("ingesting.utils")
    ret = import_pkg("retriever.utils")
    monkeypatch.setattr(utils.Config, "INDEX_SHARDS", 3)
    ix = utils.get_index("multi-shard-test", capacity=100)
    assert ix.shard_set.n == 3
    rng = np.random.default_rng(4)
    X, items = _items(rng, 200, 768)
    ix.upsert(items)
    assert ret.search(ix, X[150].tolist(), top_k=5)[0] == "v150"


def test_persistence_across_shard_counts(idxmod, cuda, tmp_path):
    rng = np.random.default_rng(5)
    a = idxmod.Index("p", dimension=512, dtype="bfloat16", capacity=1000, device=cuda, shards=3)
    X, items = _items(rng, 1000, 512)
    a.upsert(items)
    Q = rng.standard_normal((4, 512)).astype(np.float32)
    before = a.query_batch(Q, top_k=20, include_metadata=True)
    a.save(str(tmp_path / "snap"))
    for shards in (1, 2, 5):  # the snapshot is in global row order: any shard count restores it
        b = idxmod.Index.load(str(tmp_path / "snap"), device=cuda, shards=shards)
        assert b.query_batch(Q, top_k=20, include_metadata=True) == before
        b.close()
    a.close()


# ------------------------------------------------- world-2, real HIP shards --
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_worker(rank, world, port, n, result_q):
    import sys

    sys.path.insert(0, REPO)
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sharded = import_pkg("sharded")
        rng = np.random.default_rng(9)
        X = rng.standard_normal((max(n, 1), 512)).astype(np.float32)[:n]
        Q = rng.standard_normal((16, 512)).astype(np.float32)
        if n > 40:
            X[40] = X[3]
            Q[0] = X[3]
        idx = sharded.ShardedIndex(512, dtype="float16", capacity_per_rank=5000, device=0)
        if n:
            idx.upsert_rows(torch.from_numpy(X).cuda(), torch.arange(n))
        out = {}
        for mode in ("scan", "mfma"):
            s, r = idx.search(torch.from_numpy(Q).cuda(), 20, mode=mode)
            out[mode] = (s.cpu().numpy(), r.cpu().numpy())
        result_q.put((rank, idx.n_local, out))
        idx.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [3000, 1])
def test_world2_real_shards_equal_single_index(idxmod, cuda, n):
    """Two ranks (processes) with real HIP shards on the one GPU, gloo exchange; n = 1 leaves
    rank 1's shard empty.  Both ranks must return what one DeviceIndex over all rows returns."""
    import torch
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(9)
    X = rng.standard_normal((max(n, 1), 512)).astype(np.float32)[:n]
    Q = rng.standard_normal((16, 512)).astype(np.float32)
    if n > 40:
        X[40] = X[3]
        Q[0] = X[3]
    single = idxmod.DeviceIndex(512, dtype="float16", capacity=5000, device=cuda)
    single.upsert_rows(torch.from_numpy(X), torch.arange(n))
    s_ref, r_ref = single.search(torch.from_numpy(Q), 20, n, mode="scan")
    s_ref, r_ref = s_ref.cpu().numpy(), r_ref.cpu().numpy()
    assert sorted(o[1] for o in outs) == sorted([len(range(0, n, 2)), len(range(1, n, 2))])
    for rank, n_local, out in outs:
        for mode, (s, r) in out.items():
            assert np.array_equal(r, r_ref), (rank, mode)
            assert np.array_equal(s, s_ref), (rank, mode)
    if n > 40:
        assert r_ref[0, :2].tolist() == [3, 40]
    single.close()


def test_search_image_steady_state_allocates_nothing_and_fetches_once(cuda, monkeypatch):
    """/search_image over a multi-shard index (reference retriever/main.py:104-169): once the
    workspaces exist, a request makes no device / pinned allocation in the library
    (rc_alloc_count), and the search's include_values (retriever/utils.py:62-64) comes back
    with the query itself (one rc_sharded_query_host call per request) and serves the
    handler's fetch(ids) (retriever/main.py:142): no second device read."""
    import io

    from fastapi.testclient import TestClient
    from PIL import Image

    L = import_pkg("_lib")
    lib = L.load()
    utils = import_pkg("ingesting.utils")
    main = import_pkg("retriever.main")
    idxmod = import_pkg("index")
    monkeypatch.setattr(utils.Config, "INDEX_SHARDS", 3)
    ix = utils.get_index("alloc-free-search", capacity=64)
    monkeypatch.setattr(main, "index", lambda: ix)
    rng = np.random.default_rng(8)
    imgs = [rng.integers(0, 256, (224, 224, 3), dtype=np.uint8) for _ in range(6)]
    blobs = []
    for a in imgs:
        b = io.BytesIO()
        Image.fromarray(a).save(b, format="PNG")
        blobs.append(b.getvalue())
    for i, b in enumerate(blobs):
        ix.upsert([(f"img-{i}", main.get_feature_vector(b), {"gcs_path": f"images/img-{i}.png"})])
    client = TestClient(main.app)
    fetches, queries = [], []
    real_fetch, real_query = idxmod.ShardSet.fetch_rows, idxmod.ShardSet.query_host
    monkeypatch.setattr(idxmod.ShardSet, "fetch_rows",
                        lambda self, rows, stored=False: fetches.append(len(rows)) or real_fetch(self, rows, stored))
    monkeypatch.setattr(idxmod.ShardSet, "query_host",
                        lambda self, q, k, n, v: queries.append((k, v)) or real_query(self, q, k, n, v))
    first = client.post("/search_image", files={"file": ("q.png", blobs[2], "image/png")})
    assert first.status_code == 200 and first.json()[0].endswith("images/img-2.png")
    client.post("/search_image", files={"file": ("q.png", blobs[3], "image/png")})  # warm
    fetches.clear()
    queries.clear()
    n0 = lib.rc_alloc_count()
    for b in blobs:
        r = client.post("/search_image", files={"file": ("q.png", b, "image/png")})
        assert r.status_code == 200 and len(r.json()) == 5
    assert lib.rc_alloc_count() == n0
    assert queries == [(5, True)] * len(blobs) and fetches == []  # values came with the query
    ix.close()


@pytest.mark.parametrize("shards,n", [(1, 700), (3, 700), (1, 3), (3, 2)])
def test_query_host_equals_search_plus_fetch(cuda, shards, n):
    """rc_sharded_query_host (host in / host out, values gathered with the lists) returns what
    rc_sharded_search + rc_sharded_fetch return, bit for bit, including indexes smaller than k
    (-1 rows, NaN values) and an empty index; the Index query built on it matches too."""
    import torch

    idxmod = import_pkg("index")
    ss = idxmod.ShardSet(96, dtype="float16", capacity_per_shard=1024, devices=[0] * shards)
    g = torch.Generator().manual_seed(n + shards)
    X = torch.randn(n, 96, generator=g)
    ss.upsert_rows(X, torch.arange(n))
    q = torch.randn(4, 96, generator=g)
    q[1] = X[n // 2]
    for k in (1, 5, 17):
        sc, rw, val = ss.query_host(q.numpy().copy(), k, n, True)
        s_ref, r_ref = ss.search(q, k, n)
        assert np.array_equal(sc, s_ref.cpu().numpy()) and np.array_equal(rw, r_ref.cpu().numpy())
        for qi in range(4):
            for j in range(k):
                if rw[qi, j] < 0:
                    assert np.isnan(val[qi, j]).all()
                else:
                    assert np.array_equal(val[qi, j], ss.fetch_rows([int(rw[qi, j])])[0].numpy())
        sc2, rw2, v2 = ss.query_host(q.numpy().copy(), k, n, False)
        assert np.array_equal(sc2, sc) and np.array_equal(rw2, rw) and v2 is None
    e_s, e_r, _ = ss.query_host(q.numpy().copy(), 3, 0, True)
    assert np.isneginf(e_s).all() and (e_r == -1).all()
    ss.close()


@pytest.mark.parametrize("dtype,dim,n", [("float32", 768, 10000), ("float16", 96, 700), ("bfloat16", 300, 70000),
                                         ("float32", 768, 1), ("float16", 512, 33)])
def test_single_query_launch_equals_multi_kernel(cuda, dtype, dim, n):
    """One query through rc_sharded_query_host is ONE launch (query1_kernel: the query in its
    arguments, normalise + scan + last-block merge + value gather, results written into pinned
    memory); it returns the multi-kernel path's scores, rows and values bit for bit (search +
    fetch), for every storage dtype, indexes smaller than k, and back-to-back calls (the
    last-block ticket resets itself)."""
    import torch

    idxmod = import_pkg("index")
    ss = idxmod.ShardSet(dim, dtype=dtype, capacity_per_shard=max(n, 64), devices=[0])
    g = torch.Generator().manual_seed(dim + n)
    X = torch.randn(n, dim, generator=g)
    ss.upsert_rows(X, torch.arange(n))
    q = torch.randn(3, dim, generator=g)
    q[1] = X[n // 2]
    for k in (1, 5, 100):
        for qi in range(3):
            for rep in range(2):
                sc, rw, val = (a.copy() for a in ss.query_host(q[qi:qi + 1].numpy().copy(), k, n, True))
                s_ref, r_ref = ss.search(q[qi:qi + 1], k, n)
                assert np.array_equal(sc, s_ref.cpu().numpy()), (k, qi, rep)
                assert np.array_equal(rw, r_ref.cpu().numpy()), (k, qi, rep)
                live = rw[0] >= 0
                assert live.sum() == min(k, n)
                if live.any():
                    want = ss.fetch_rows([int(r) for r in rw[0][live]]).numpy()
                    assert np.array_equal(val[0][live], want)
                assert np.isnan(val[0][~live]).all()
    sc1, rw1, v1 = ss.query_host(q[1:2].numpy().copy(), 5, n, False)
    assert rw1[0, 0] == n // 2 and v1 is None
    ss.close()
