"""World-size-2 (and 4) gloo test of the sharded search orchestration on CPU.

The per-shard scan and the device merge are HIP kernels (covered by -m gpu tests,
including a world-2 run over real HIP shards in test_sharded_gpu.py); here they
are replaced by the CPU oracle so the distributed plumbing — round-robin row
ownership, upsert routing, empty shards, all_gather of (score, global row) lists,
merge order across ranks — is checked end to end with real torch.distributed
collectives.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO, import_pkg


class OracleShard:
    """CPU stand-in for DeviceIndex: stores normalised rows, exact float64 top-k,
    returns global rows row_base + local * row_stride; an empty shard answers -inf / -1."""

    def __init__(self, dim, capacity, row_base, row_stride):
        self.X = np.zeros((capacity, dim))
        self.row_base = row_base
        self.row_stride = row_stride

    def upsert_rows(self, vecs, rows):
        v = vecs.double().numpy()
        self.X[rows.numpy()] = v / np.linalg.norm(v, axis=1, keepdims=True)

    def search(self, queries, k, n_rows):
        from oracle.cosine_topk import cosine_topk

        nq = queries.shape[0]
        if n_rows == 0:
            return torch.full((nq, k), -float("inf")), torch.full((nq, k), -1, dtype=torch.int64)
        r, s = cosine_topk(self.X[:n_rows], queries.double().numpy(), k, rows_normalized=True)
        r = r * self.row_stride + self.row_base
        pad = k - r.shape[1]
        if pad > 0:
            r = np.pad(r, ((0, 0), (0, pad)), constant_values=-1)
            s = np.pad(s, ((0, 0), (0, pad)), constant_values=-np.inf)
        return torch.from_numpy(s.astype(np.float32)), torch.from_numpy(r)


def cpu_merge(gs, gr, k):
    """Restates rc_topk_merge on CPU: key (score desc, global row asc), empty slots (row < 0) dropped."""
    W, nq, kin = gs.shape
    out_s = torch.full((nq, k), -float("inf"))
    out_r = torch.full((nq, k), -1, dtype=torch.int64)
    for q in range(nq):
        cand = sorted((-float(gs[w, q, t]), int(gr[w, q, t])) for w in range(W) for t in range(kin) if gr[w, q, t] >= 0)
        for j, (negs, row) in enumerate(cand[:k]):
            out_s[q, j] = -negs
            out_r[q, j] = row
    return out_s, out_r


def _data(world, n):
    cap, dim = 300, 64
    rng = np.random.default_rng(0)  # same data on every rank
    X = rng.standard_normal((n, dim)).astype(np.float32)
    Q = rng.standard_normal((3, dim)).astype(np.float32)
    if n > cap + 11:
        X[5] = X[cap + 11]  # an exact tie across shards (5 % W != (cap + 11) % W for W = 2, 4)
        Q[0] = X[cap + 11]
    return X, Q


def _worker(rank, world, n, port, result_q):
    import sys

    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sharded = import_pkg("sharded")
        cap, dim, k = 300, 64, 7
        idx = sharded.ShardedIndex(dim, capacity_per_rank=cap,
                                   backend_factory=lambda: OracleShard(dim, cap, rank, world), merge_fn=cpu_merge)
        X, Q = _data(world, n)
        owned = idx.upsert_rows(torch.from_numpy(X), torch.arange(n))
        s, r = idx.search(torch.from_numpy(Q), k)
        result_q.put((rank, owned, idx.n_local, s.numpy(), r.numpy()))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,n", [(2, 550), (4, 1150), (4, 2), (2, 1)])
def test_sharded_search_equals_global_oracle(world, n):
    """Round-robin shards + all_gather + merge == one exact index; n < world leaves ranks with
    EMPTY shards, which must still answer (-inf, -1) lists and reach the collective."""
    from oracle.cosine_topk import cosine_topk

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, n, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cap, k = 300, 7
    X, Q = _data(world, n)
    ref_r, ref_s = cosine_topk(X, Q, k)
    kk = min(k, n)
    assert sum(o[1] for o in outs) == n  # every row written by exactly one owner
    for rank, owned, n_local, s, r in outs:
        assert owned == n_local == len(range(rank, n, world))  # round-robin: rank r owns rows r, r+W, ...
        assert np.array_equal(r[:, :kk], ref_r), (rank, r, ref_r)  # identical on every rank
        assert np.allclose(s[:, :kk], ref_s, atol=1e-6)
        assert np.all(r[:, kk:] == -1) and np.all(np.isneginf(s[:, kk:]))
    if n > cap + 11:
        assert outs[0][4][0, :2].tolist() == [5, cap + 11]  # tie → lower global row first


def _worker_local(rank, world, counts, port, result_q):
    import sys

    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sharded = import_pkg("sharded")
        cap, dim, k = 300, 64, 5
        idx = sharded.ShardedIndex(dim, capacity_per_rank=cap,
                                   backend_factory=lambda: OracleShard(dim, cap, rank, world), merge_fn=cpu_merge)
        X, Q = _data(world, cap * world)
        mine = X[rank::world][:counts[rank]]  # rank r's local row j is global row j * W + r
        idx.upsert_local(torch.from_numpy(mine), torch.arange(counts[rank]))
        errors = []
        try:
            idx.upsert_local(torch.from_numpy(mine[:1]), torch.tensor([cap]))
        except ValueError:
            errors.append("capacity")
        try:
            idx.set_rows(world * (counts[rank] + 1))
        except ValueError:
            errors.append("set_rows")
        n_rows = idx.publish_rows()
        s, r = idx.search(torch.from_numpy(Q), k)
        result_q.put((rank, n_rows, errors, s.numpy(), r.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,counts", [(2, (40, 37)), (4, (10, 12, 9, 11))])
def test_rank_local_ingest_publishes_consistent_rows(world, counts):
    """Data-parallel ingest (upsert_local per rank, no collective) with UNEVEN per-rank counts:
    publish_rows agrees on the largest global range every shard covers (min_r written_r*W + r),
    the search over it equals one exact index; out-of-capacity rows and an over-long set_rows
    are rejected instead of exposing unwritten (zero) rows as matches."""
    from oracle.cosine_topk import cosine_topk

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_local, args=(r, world, counts, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = min(c * world + r for r, c in enumerate(counts))
    X, Q = _data(world, 300 * world)
    ref_r, ref_s = cosine_topk(X[:want], Q, 5)
    for rank, n_rows, errors, s, r in outs:
        assert n_rows == want
        assert errors == ["capacity", "set_rows"]
        assert np.array_equal(r, ref_r)
        assert np.allclose(s, ref_s, atol=1e-6)


def test_row_coverage_counts_only_the_gap_free_prefix():
    """upsert_local of local rows 0-9 then 20-29 leaves a hole: written stays 10 and set_rows
    refuses a range over the hole; filling 10-19 closes it (written was a high-water
    mark that accepted the zero rows)."""
    sharded = import_pkg("sharded")
    cap, dim = 64, 8
    idx = sharded.ShardedIndex(dim, capacity_per_rank=cap, backend_factory=lambda: OracleShard(dim, cap, 0, 1),
                               merge_fn=cpu_merge)
    X = torch.randn(40, dim)
    idx.upsert_local(X[:10], torch.arange(10))
    idx.upsert_local(X[20:30], torch.arange(20, 30))
    assert idx.written == 10 and idx.coverage.runs == [[0, 10], [20, 30]]
    with pytest.raises(ValueError):
        idx.set_rows(30)
    idx.set_rows(10)
    idx.upsert_local(X[10:20], torch.tensor([19, 10, 11, 12, 13, 14, 15, 16, 17, 18]))
    assert idx.written == 30 and idx.coverage.runs == [[0, 30]]
    assert idx.publish_rows() == 30
    idx.upsert_rows(X[:3], torch.tensor([35, 33, 33]))  # scattered, repeated rows
    assert idx.coverage.runs == [[0, 30], [33, 34], [35, 36]] and idx.written == 30
    cov = sharded.RowCoverage()
    for lo, hi in [(5, 7), (0, 2), (2, 5), (9, 10)]:
        cov.add(lo, hi)
    assert cov.runs == [[0, 7], [9, 10]] and cov.prefix == 7
