"""World-size-2 (and 4) gloo test of the sharded search orchestration on CPU.

The per-shard scan and the device merge are HIP kernels (covered by -m gpu tests);
here they are replaced by the CPU oracle so the distributed plumbing — row
ownership, upsert routing, all_gather of (score, global row) lists, merge order
across ranks — is checked end to end with real torch.distributed collectives.
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
    """CPU stand-in for DeviceIndex: stores normalised rows, exact float64 top-k."""

    def __init__(self, dim, capacity, row_base):
        self.X = np.zeros((capacity, dim))
        self.row_base = row_base

    def upsert_rows(self, vecs, rows):
        v = vecs.double().numpy()
        self.X[rows.numpy()] = v / np.linalg.norm(v, axis=1, keepdims=True)

    def search(self, queries, k, n_rows):
        from oracle.cosine_topk import cosine_topk

        r, s = cosine_topk(self.X[:n_rows], queries.double().numpy(), k, rows_normalized=True)
        pad = k - r.shape[1]
        if pad > 0:
            r = np.pad(r, ((0, 0), (0, pad)), constant_values=-1 - self.row_base)
            s = np.pad(s, ((0, 0), (0, pad)), constant_values=-np.inf)
        return torch.from_numpy(s.astype(np.float32)), torch.from_numpy(r + self.row_base)


def cpu_merge(gs, gr, k):
    """Restates rc_topk_merge on CPU: key (score desc, list position asc), invalid rows dropped."""
    W, nq, kin = gs.shape
    out_s = torch.full((nq, k), -float("inf"))
    out_r = torch.full((nq, k), -1, dtype=torch.int64)
    for q in range(nq):
        cand = [(-float(gs[w, q, t]), w * kin + t) for w in range(W) for t in range(kin) if gr[w, q, t] >= 0]
        cand.sort()
        for j, (negs, pos) in enumerate(cand[:k]):
            out_s[q, j] = -negs
            out_r[q, j] = gr[pos // kin, q, pos % kin]
    return out_s, out_r


def _worker(rank, world, port, result_q):
    import sys

    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sharded = import_pkg("sharded")
        cap, dim, k = 300, 64, 7
        idx = sharded.ShardedIndex(dim, capacity_per_rank=cap,
                                   backend_factory=lambda: OracleShard(dim, cap, rank * cap), merge_fn=cpu_merge)
        rng = np.random.default_rng(0)  # same data on every rank
        n = cap * world - 50
        X = rng.standard_normal((n, dim)).astype(np.float32)
        X[5] = X[cap + 11]  # cross-shard exact tie
        Q = rng.standard_normal((3, dim)).astype(np.float32)
        Q[0] = X[cap + 11]
        owned = idx.upsert_rows(torch.from_numpy(X), torch.arange(n))
        s, r = idx.search(torch.from_numpy(Q), k)
        result_q.put((rank, owned, s.numpy(), r.numpy()))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_search_equals_global_oracle(world):
    from oracle.cosine_topk import cosine_topk

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cap, dim, k = 300, 64, 7
    rng = np.random.default_rng(0)
    n = cap * world - 50
    X = rng.standard_normal((n, dim)).astype(np.float32)
    X[5] = X[cap + 11]
    Q = rng.standard_normal((3, dim)).astype(np.float32)
    Q[0] = X[cap + 11]
    ref_r, ref_s = cosine_topk(X, Q, k)
    assert sum(o[1] for o in outs) == n  # every row written by exactly one owner
    for rank, owned, s, r in outs:
        assert np.array_equal(r, ref_r), (rank, r, ref_r)  # identical on every rank
        assert np.allclose(s, ref_s, atol=1e-6)
    assert outs[0][3][0, :2].tolist() == [5, cap + 11]  # tie → lower global row first
