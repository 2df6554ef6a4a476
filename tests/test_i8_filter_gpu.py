"""GPU parity of the batched search with the int8 filter copy (rc_index_set_filter(RC_FILTER_I8)).

Reference path replaced: Pinecone ``index.query`` (``retriever/utils.py:59-66``) for a batch
of query vectors, as in tests/test_batched_search_gpu.py.  The int8 copy only decides which
rows are rescored; the rescoring is the single-query scan's f32 arithmetic on the stored
rows, so the bar is the same: the MFMA path returns EXACTLY (bit for bit) what the scan
returns, and the scan matches the float64 oracle (tests/test_batched_search_gpu.py).  A row
the int8 filter wrongly dropped (a bound that does not hold) would show up as a diff.  The
cases cover every way the copy is written (upsert, overwrite, fill, import, grow, enabling
on a populated index), row shapes that stress the per-row scale (one-hot rows, one massive
channel, tiny rows), exact ties that overflow the candidate lists, and the f32 index (the
copy makes the batched path available there).
"""
import numpy as np
import pytest

from conftest import import_pkg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def idxmod(cuda):
    return import_pkg("index")


def _same(dev, Q, k, n):
    import torch

    s_m, r_m = dev.search(Q, k, n, mode="mfma")
    s_s, r_s = dev.search(Q, k, n, mode="scan")
    torch.cuda.synchronize()
    assert torch.equal(r_m, r_s), "int8-filtered batched search and scan disagree on rows"
    assert torch.equal(s_m, s_s), "int8-filtered batched search and scan disagree on scores"
    return s_m, r_m


@pytest.mark.parametrize("dtype", ["float16", "bfloat16", "float32"])
@pytest.mark.parametrize("dim", [512, 200, 768])
@pytest.mark.parametrize("n,k,nq", [(200, 5, 3), (5000, 10, 1), (70_000, 100, 20), (70_000, 256, 9), (300_000, 10, 300)])
def test_i8_filter_matches_scan(idxmod, cuda, dtype, dim, n, k, nq):
    import torch

    rng = np.random.default_rng(n + dim + k + nq)
    X = rng.standard_normal((n, dim)).astype(np.float32)
    Q = rng.standard_normal((nq, dim)).astype(np.float32)
    Q[0] = X[n // 3]
    dev = idxmod.DeviceIndex(dim, dtype=dtype, capacity=n, device=cuda)
    dev.upsert_rows(torch.from_numpy(X), torch.arange(n, dtype=torch.int64))
    dev.set_filter("i8")
    assert dev.filter == "i8"
    _, r = _same(dev, torch.from_numpy(Q), k, n)
    assert int(r[0, 0]) == n // 3
    dev.close()


def test_i8_copy_follows_every_write(idxmod, cuda):
    """Enabled on an empty index, then: upsert, overwrite, fill_random, grow, import — each
    write path must refresh the copy, or the filter would score stale rows."""
    import torch

    dim, n0 = 512, 40_000
    rng = np.random.default_rng(7)
    dev = idxmod.DeviceIndex(dim, dtype="float16", capacity=n0, device=cuda)
    dev.set_filter("i8")
    X = rng.standard_normal((n0, dim)).astype(np.float32)
    dev.upsert_rows(torch.from_numpy(X), torch.arange(n0))
    Q = torch.from_numpy(rng.standard_normal((24, dim)).astype(np.float32))
    _same(dev, Q, 20, n0)
    # overwrite rows to be the queries themselves: they must now come first
    hit = torch.tensor([5, 17_000, 39_999])
    dev.upsert_rows(Q[:3], hit)
    _, r = _same(dev, Q, 20, n0)
    assert r[:3, 0].cpu().tolist() == hit.tolist()
    # grow (copy moves with the rows), then fill the new range
    dev.grow(100_000)
    dev.fill_random(3, n0, 60_000)
    _, r = _same(dev, Q, 20, 100_000)
    assert r[:3, 0].cpu().tolist() == hit.tolist()
    # import raw rows over [0, 1000) from another index
    src = idxmod.DeviceIndex(dim, dtype="float16", capacity=1000, device=cuda)
    src.fill_random(9, 0, 1000)
    rows, norms = src.export_rows(0, 1000)
    dev.import_rows(0, rows, norms)
    q2 = src.stored_rows(torch.tensor([0, 500, 999]))
    _, r = _same(dev, torch.cat([q2.cpu(), Q]), 20, 100_000)
    assert r[:3, 0].cpu().tolist() == [0, 500, 999]
    # off and on again: same results
    dev.set_filter("native")
    assert dev.filter == "native"
    s_n, r_n = dev.search(Q, 20, 100_000, mode="mfma")
    dev.set_filter("i8")
    s_i, r_i = dev.search(Q, 20, 100_000, mode="mfma")
    assert torch.equal(r_n, r_i) and torch.equal(s_n, s_i)
    src.close()
    dev.close()


@pytest.mark.parametrize("shape", ["one_hot", "massive_channel", "tiny_rows", "sparse"])
def test_i8_bound_holds_on_adversarial_rows(idxmod, cuda, shape):
    """Rows whose per-row scale is set by one large component quantise the rest coarsely:
    the residual norm ex grows and the filter keeps more candidates, but never drops one."""
    import torch

    n, dim = 80_000, 512
    rng = np.random.default_rng(11)
    X = rng.standard_normal((n, dim)).astype(np.float32)
    if shape == "one_hot":
        X[: n // 2] = 0
        X[np.arange(n // 2), rng.integers(0, dim, n // 2)] = 1.0
    elif shape == "massive_channel":
        X[:, 3] *= 300.0
    elif shape == "tiny_rows":
        X *= 1e-15  # normalised anyway: scale must not matter
    else:
        X[rng.random((n, dim)) < 0.97] = 0
        X[X.sum(axis=1) == 0, 0] = 1.0
    Q = rng.standard_normal((40, dim)).astype(np.float32)
    Q[:4] = X[[1, 2, n // 2 + 1, n - 1]]
    dev = idxmod.DeviceIndex(dim, dtype="float16", capacity=n, device=cuda)
    dev.upsert_rows(torch.from_numpy(X), torch.arange(n))
    dev.set_filter("i8")
    _same(dev, torch.from_numpy(Q), 50, n)
    dev.close()


def test_i8_duplicate_rows_fall_back_exactly(idxmod, cuda):
    import torch

    rng = np.random.default_rng(3)
    base = rng.standard_normal((3, 512)).astype(np.float32)
    n = 100_000
    X = base[rng.integers(0, 3, n)]
    dev = idxmod.DeviceIndex(512, dtype="float16", capacity=n, device=cuda)
    dev.upsert_rows(torch.from_numpy(X), torch.arange(n))
    dev.set_filter("i8")
    Q = torch.from_numpy(np.concatenate([base[:2], rng.standard_normal((14, 512)).astype(np.float32)]))
    dev.timing(True)
    _same(dev, Q, 50, n)
    assert dev.gemm_timing_read()[3] >= 1
    dev.timing(False)
    dev.close()


def test_i8_sublaunches_and_query_blocks(idxmod, cuda):
    """9M x 256 rows (two 2-GB int8 sub-launches per late stage) and 700 queries (3 query blocks)."""
    import torch

    n, dim, nq = 9_000_000, 256, 700
    d = idxmod.DeviceIndex(dim, dtype="float16", capacity=n, device=0)
    d.fill_random(21, 0, n)
    d.set_filter("i8")
    g = torch.Generator(device="cuda").manual_seed(22)
    q = torch.randn((nq, dim), device="cuda", generator=g)
    d.timing(True)
    _same(d, q, 100, n)
    assert d.gemm_timing_read()[3] == 0  # random data: no candidate overflow
    d.timing(False)
    d.close()


def test_i8_unsupported_width_and_bad_kind(idxmod, cuda):
    dev = idxmod.DeviceIndex(1000, dtype="float16", capacity=1000, device=cuda)  # ld 1024
    with pytest.raises(ValueError):
        dev.set_filter("i8")
    with pytest.raises(ValueError):
        dev.set_filter("fp4")
    assert dev.filter == "native"
    dev.close()


def test_i8_sharded_index_and_snapshot(idxmod, cuda, tmp_path):
    """Index(filter="i8") over 3 shards on one GPU: batched queries equal the scan; the
    snapshot remembers the filter."""
    import torch

    rng = np.random.default_rng(5)
    idx = idxmod.Index("i8", dimension=512, dtype="float16", capacity=30_000, shards=3, device=cuda, filter="i8")
    X = rng.standard_normal((30_000, 512)).astype(np.float32)
    idx.upsert_tensor([f"v{i}" for i in range(30_000)], torch.from_numpy(X).cuda())
    Q = torch.from_numpy(rng.standard_normal((64, 512)).astype(np.float32))
    ss = idx.shard_set
    s1, r1 = ss.search(Q, 30, 30_000, mode="mfma")
    s2, r2 = ss.search(Q, 30, 30_000, mode="scan")
    assert torch.equal(r1, r2) and torch.equal(s1, s2)
    idx.save(str(tmp_path / "snap"))
    idx2 = idxmod.Index.load(str(tmp_path / "snap"), device=cuda)
    assert idx2.shard_set.filter == "i8"
    s3, r3 = idx2.shard_set.search(Q, 30, 30_000, mode="mfma")
    assert torch.equal(r1, r3) and torch.equal(s1, s3)
    idx.close()
    idx2.close()
