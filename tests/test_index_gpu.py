"""GPU parity of the exact cosine index (HIP scan + wavefront top-k) against the oracle.

Reference path replaced: Pinecone ``index.query`` (``retriever/utils.py:59-66``)
and ``index.upsert`` (``ingesting/main.py:156-158``).  Bar (north star):
top-k sets identical except ties within 1e-5 score; scores within 1e-5 of the
float64 oracle run on the SAME stored (normalised, dtype-rounded) rows.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, import_pkg
from oracle.cosine_topk import cosine_topk, planted_index, topk_equal_modulo_ties

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def idxmod(cuda):
    return import_pkg("index")


def _check(dev, X_stored, Q, k, got_s, got_r, tol=1e-5):
    ref_r, ref_s = cosine_topk(X_stored, Q, k, rows_normalized=True)
    got_s = got_s.cpu().numpy()
    got_r = got_r.cpu().numpy()
    n = X_stored.shape[0]
    kk = min(k, n)
    for q in range(Q.shape[0]):
        assert topk_equal_modulo_ties(got_r[q, :kk], got_s[q, :kk], ref_r[q], ref_s[q], tol), (q, got_r[q, :kk], ref_r[q])
        # scores agree with the oracle's score of the row the kernel returned
        Xq = X_stored[got_r[q, :kk]].astype(np.float64)
        qn = Q[q].astype(np.float64) / np.linalg.norm(Q[q].astype(np.float64))
        assert np.allclose(got_s[q, :kk], Xq @ qn, atol=tol, rtol=0)
        assert np.all(np.diff(got_s[q, :kk]) <= 0), "scores not descending"
        if k > n:
            assert np.all(got_r[q, n:] == -1) and np.all(np.isneginf(got_s[q, n:]))


@pytest.mark.parametrize("dtype", ["float32", "float16", "bfloat16"])
@pytest.mark.parametrize("dim", [512, 768, 100])
@pytest.mark.parametrize("n,k,nq", [(1, 5, 1), (37, 10, 3), (1000, 10, 1), (5000, 100, 2), (20000, 5, 4), (3000, 256, 1)])
def test_search_matches_oracle(idxmod, cuda, dtype, dim, n, k, nq):
    import torch

    rng = np.random.default_rng(n * 7 + dim + k)
    X = rng.standard_normal((n, dim)).astype(np.float32)
    Q = rng.standard_normal((nq, dim)).astype(np.float32)
    dev = idxmod.DeviceIndex(dim, dtype=dtype, capacity=n + 3, device=cuda)
    dev.upsert_rows(torch.from_numpy(X), torch.arange(n, dtype=torch.int64))
    s, r = dev.search(torch.from_numpy(Q), k, n)
    torch.cuda.synchronize()
    Xs = dev.stored_rows(n).cpu().numpy()
    # stored rows are the normalised rows rounded to the storage dtype
    Xn = X / np.linalg.norm(X, axis=1, keepdims=True)
    atol = {"float32": 1e-6, "float16": 1e-3, "bfloat16": 8e-3}[dtype]
    assert np.allclose(Xs, Xn, atol=atol)
    _check(dev, Xs, Q, k, s, r)
    dev.close()


def test_exact_ties_row_ascending(idxmod, cuda):
    """Duplicate rows score identically: the tie rule (score desc, row asc) must hold exactly."""
    import torch

    rng = np.random.default_rng(3)
    base = rng.standard_normal((4, 512)).astype(np.float32)
    X = base[rng.integers(0, 4, 3000)]
    dev = idxmod.DeviceIndex(512, capacity=3000, device=cuda)
    dev.upsert_rows(torch.from_numpy(X), torch.arange(3000))
    q = base[1:2] + 0.01 * rng.standard_normal((1, 512)).astype(np.float32)
    s, r = dev.search(torch.from_numpy(q), 64, 3000)
    ref_r, _ = cosine_topk(dev.stored_rows(3000).cpu().numpy(), q, 64, rows_normalized=True)
    assert r.cpu().numpy()[0].tolist() == ref_r[0].tolist()


def test_golden_planted_top5(idxmod, cuda):
    """Config 1's index: seeded 10k x 768 rows + planted near-duplicates of the test-image embedding."""
    import torch

    sys_path_golden = GOLDEN
    g = json.load(open(os.path.join(sys_path_golden, "golden.json")))
    emb = np.load(os.path.join(sys_path_golden, "test_image_embedding_seed1907.npy"))
    X, planted = planted_index(emb)
    dev = idxmod.DeviceIndex(768, capacity=X.shape[0], device=cuda)
    dev.upsert_rows(torch.from_numpy(X), torch.arange(X.shape[0]))
    s, r = dev.search(torch.from_numpy(emb[None]), 5, X.shape[0])
    assert r.cpu().numpy()[0].tolist() == g["top5_rows"]
    assert np.allclose(s.cpu().numpy()[0], g["top5_scores"], atol=1e-5)


def test_upsert_overwrites_and_fetch(idxmod, cuda):
    import torch

    rng = np.random.default_rng(5)
    X = rng.standard_normal((10, 768)).astype(np.float32)
    dev = idxmod.DeviceIndex(768, capacity=16, device=cuda)
    dev.upsert_rows(torch.from_numpy(X), torch.arange(10))
    Y = rng.standard_normal((2, 768)).astype(np.float32)
    dev.upsert_rows(torch.from_numpy(Y), torch.tensor([3, 7]))
    X[3], X[7] = Y[0], Y[1]
    got = dev.fetch_rows(torch.arange(10)).cpu().numpy()
    assert np.allclose(got, X, rtol=1e-5, atol=1e-5)
    s, r = dev.search(torch.from_numpy(Y[1:2]), 1, 10)
    assert int(r[0, 0]) == 7 and abs(float(s[0, 0]) - 1.0) < 1e-5


def _splitmix64(x):
    x = (x + np.uint64(0x9E3779B97F4A7C15))
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


@pytest.mark.parametrize("dtype", ["float32", "float16"])
def test_fill_random_matches_numpy(idxmod, cuda, dtype):
    import torch

    n, dim, seed = 300, 512, 4
    dev = idxmod.DeviceIndex(dim, dtype=dtype, capacity=n, device=cuda)
    dev.fill_random(seed, 0, n)
    got = dev.stored_rows(n).cpu().numpy()
    with np.errstate(over="ignore"):
        rr = np.arange(n, dtype=np.uint64)[:, None]
        cc = np.arange(dim, dtype=np.uint64)[None, :]
        h = _splitmix64(np.uint64(seed) * np.uint64(0xD1342543DE82EF95) + rr * np.uint64(dim) + cc)
    v = (h >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 8388608.0) - np.float32(1.0)
    v = v / np.linalg.norm(v.astype(np.float64), axis=1, keepdims=True)
    assert np.allclose(got, v, atol=1e-6 if dtype == "float32" else 1e-3)


def test_cross_shard_merge_equals_single_index(idxmod, cuda):
    """Four shards (row_base offsets) + rc_topk_merge == one index over all rows."""
    import torch

    rng = np.random.default_rng(11)
    n_per, dim, k, nq = 2500, 512, 50, 3
    X = rng.standard_normal((4 * n_per, dim)).astype(np.float32)
    X[1234] = X[7777]  # a cross-shard exact tie
    Q = rng.standard_normal((nq, dim)).astype(np.float32)
    Q[0] = X[7777]
    ss, rs, stored = [], [], []
    for sh in range(4):
        d = idxmod.DeviceIndex(dim, capacity=n_per, device=cuda, row_base=sh * n_per)
        d.upsert_rows(torch.from_numpy(X[sh * n_per:(sh + 1) * n_per]), torch.arange(n_per))
        s, r = d.search(torch.from_numpy(Q), k, n_per)
        ss.append(s)
        rs.append(r)
        stored.append(d.stored_rows(n_per).cpu().numpy())
    ms, mr = idxmod.topk_merge(torch.stack(ss), torch.stack(rs), k)
    Xs = np.concatenate(stored)
    ref_r, ref_s = cosine_topk(Xs, Q, k, rows_normalized=True)
    for q in range(nq):
        assert topk_equal_modulo_ties(mr[q].cpu().numpy(), ms[q].cpu().numpy(), ref_r[q], ref_s[q])
    assert mr[0, :2].cpu().tolist() == [1234, 7777]


def test_config3_full_size_planted(idxmod, cuda):
    """Config 3 at full size (1M x 512 f32, top-10): size-independent properties.

    Rows come from the on-device generator; query j is a copy of a known row, so
    its top-1 must be that row at score 1 (to f32 rounding), and the returned
    scores must equal the oracle's score of the returned rows."""
    import torch

    n, dim = 1_000_000, 512
    dev = idxmod.DeviceIndex(dim, capacity=n, device=cuda)
    dev.fill_random(2, 0, n)
    targets = torch.tensor([0, 123_457, 999_999], dtype=torch.int64)
    Q = dev.stored_rows(targets)
    s, r = dev.search(Q, 10, n)
    assert r[:, 0].cpu().tolist() == targets.tolist()
    assert torch.allclose(s[:, 0].cpu(), torch.ones(3), atol=2e-6)
    Xr = dev.stored_rows(r.reshape(-1)).reshape(3, 10, dim).double()
    qn = Q.double() / Q.double().norm(dim=1, keepdim=True)
    assert torch.allclose(torch.einsum("qkd,qd->qk", Xr, qn).cpu(), s.double().cpu(), atol=1e-5)


def test_query_host_values_follow_each_query(idxmod, cuda):
    """The one-shard request path (rc_sharded_query_host -> query1 launch pair writing scores, rows
    and the matches' values into reused pinned memory; the host polls a completion word the
    finishing block stores after them): alternating distinct queries with include_values=True,
    every match carries exactly its own row's upserted vector (no value left over from the
    previous query), and ids / scores equal the multi-kernel device search (rc_sharded_search)."""
    import torch

    rng = np.random.default_rng(11)
    X = rng.standard_normal((10000, 768)).astype(np.float32)
    ix = idxmod.Index("q1-values", dimension=768, dtype="float32", capacity=len(X), device=cuda)
    ix.upsert_tensor([f"r{i}" for i in range(len(X))], torch.from_numpy(X).to(cuda))
    qs = [X[i] + 0.01 * rng.standard_normal(768).astype(np.float32) for i in (5, 777, 5, 9999, 1234, 777)]
    for q in qs * 3:
        res = ix.query(vector=q.tolist(), top_k=5, include_values=True)["matches"]
        s_dev, r_dev = ix.shard_set.search(torch.from_numpy(q[None]), 5, len(ix))
        assert [m["id"] for m in res] == [f"r{r}" for r in r_dev[0].tolist()]
        assert [m["score"] for m in res] == s_dev[0].tolist()
        # the values are fetch_kernel's arithmetic (stored row x norm): the same bits as the
        # staged device fetch of those rows, within float rounding of the upserted vectors
        want = ix.shard_set.fetch_rows(r_dev[0].cpu()).numpy()
        for m, w in zip(res, want):
            v = np.asarray(m["values"], np.float32)
            assert np.array_equal(v, w), m["id"]
            assert np.allclose(v, X[int(m["id"][1:])], rtol=1e-6, atol=1e-6)
        ids = [m["id"] for m in res]
        got = ix.fetch(ids)["vectors"]  # served from the values this query just fetched
        for i, w in zip(ids, want):
            assert np.array_equal(np.asarray(got[i]["values"], np.float32), w)
    ix.close()


@pytest.mark.parametrize("n,k,cluster", [(100_000, 100, True), (32_768, 100, False), (100_000, 256, True)])
def test_merge_heads_fallback_paths(idxmod, cuda, n, k, cluster):
    """merge_heads_kernel's two rarely-taken paths, checked against the oracle: (a) the true top-k
    packed into one scan block's contiguous rows (near-duplicates ingested back to back), so the
    heads' threshold admits more than CAP candidates and the block falls back to the full merge;
    (b) fewer lists than k (64 lists of 512 rows, k = 100): the heads' k-th key is EMPTY, every key
    qualifies, and the full merge runs again."""
    import torch

    rng = np.random.default_rng(n + k)
    dim = 512
    X = rng.standard_normal((n, dim)).astype(np.float32)
    Q = rng.standard_normal((2, dim)).astype(np.float32)
    if cluster:
        r0 = 1024  # rows 1024 .. 1024 + k - 1: all inside the third 512-row scan block
        X[r0:r0 + k] = Q[0] + 0.05 * rng.standard_normal((k, dim)).astype(np.float32)
    dev = idxmod.DeviceIndex(dim, capacity=n, device=cuda)
    dev.upsert_rows(torch.from_numpy(X), torch.arange(n, dtype=torch.int64))
    s, r = dev.search(torch.from_numpy(Q), k, n)
    torch.cuda.synchronize()
    Xs = dev.stored_rows(n).cpu().numpy()
    _check(dev, Xs, Q, k, s, r)
    if cluster:
        assert sorted(r.cpu().numpy()[0].tolist()) == list(range(1024, 1024 + k))
    dev.close()
