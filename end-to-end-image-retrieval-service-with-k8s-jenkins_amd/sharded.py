"""Row-sharded exact cosine index across the GPUs of one node (one process per GPU).

SURVEY §8(e): global row g lives on rank ``g % W`` as local row ``g // W``
(round-robin routing, so every rank's shard fills from the first upsert); the
shard reports global rows itself (``rc_index_set_row_map(rank, W)``).  A query
batch (identical on every rank) is searched by each rank's HIP kernels over its
shard → local top-k ``(f32 score, i64 global row)``; one
``all_gather_into_tensor`` per output (RCCL over xGMI under the ``nccl``
backend, Q*k*12 B per rank; host tensors under ``gloo``) brings every rank's
list to every rank, and ``rc_topk_merge`` merges them on the device keyed by
(score desc, global row asc) — the order one index over all rows gives.  An
empty shard answers ``(-inf, -1)`` lists, so every rank always reaches the
collective.  Upserts need no collective: a row is written only by its owner.

Pinecone does the cross-partition merge server-side (the reference only sees
``index.query`` at ``retriever/utils.py:62``); this is the MI355X equivalent.
The single-process form (several shards driven by one process, peer copies
instead of a collective) is ``index.ShardSet`` / ``rc_sharded``.
"""
from __future__ import annotations

import json
import os
from typing import Callable

import torch
import torch.distributed as dist


class RowCoverage:
    """The local rows a shard holds, as sorted disjoint [lo, hi) runs.  ``prefix`` is the
    gap-free count: rows [0, prefix) all hold data.  Rows past a gap are tracked but never
    counted, so a row range with a hole (zero rows that would score 0 and come back as
    matches for ids that do not exist) is never published."""

    def __init__(self):
        self.runs: list[list[int]] = []

    def add(self, lo: int, hi: int) -> None:
        if hi <= lo:
            return
        keep = []
        for a, b in self.runs:
            if b < lo or a > hi:  # disjoint and not touching
                keep.append([a, b])
            else:  # overlapping or adjacent: merged into [lo, hi)
                lo, hi = min(lo, a), max(hi, b)
        keep.append([lo, hi])
        keep.sort()
        self.runs = keep

    def add_rows(self, rows: torch.Tensor) -> None:
        """Every row in ``rows`` (any order, repeats allowed, host or device)."""
        u = torch.unique(torch.as_tensor(rows).reshape(-1))
        if u.numel() == 0:
            return
        lo, hi = int(u[0]), int(u[-1])
        if hi - lo + 1 == u.numel():  # one contiguous run (the common case: no host copy of the rows)
            self.add(lo, hi + 1)
            return
        v = u.cpu().tolist()
        start = prev = v[0]
        for x in v[1:]:
            if x != prev + 1:
                self.add(start, prev + 1)
                start = x
            prev = x
        self.add(start, prev + 1)

    @property
    def prefix(self) -> int:
        return self.runs[0][1] if self.runs and self.runs[0][0] == 0 else 0


class ShardedIndex:
    def __init__(self, dim: int, dtype: str = "float16", capacity_per_rank: int = 1 << 20, group=None,
                 device=None, backend_factory: Callable | None = None, merge_fn: Callable | None = None,
                 filter: str = "native"):
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.host_exchange = dist.is_initialized() and dist.get_backend(group) == "gloo"
        self.dim = int(dim)
        self.capacity = int(capacity_per_rank)
        # global rows key the cross-rank merge in 32 bits (merge_lists_kernel): the last
        # global row, (capacity - 1) * world + rank, must stay below 2^32 - 1
        if self.capacity < 1 or (self.capacity - 1) * self.world + self.world - 1 >= (1 << 32) - 1:
            raise ValueError(f"capacity_per_rank x world = {self.capacity} x {self.world} exceeds the 2^32 - 1 "
                             "global rows the top-k merge can key")
        if backend_factory is None:
            from .index import DeviceIndex, topk_merge

            backend_factory = lambda: DeviceIndex(dim, dtype=dtype, capacity=capacity_per_rank, device=device,
                                                  row_base=self.rank, row_stride=self.world)
            merge_fn = merge_fn or topk_merge
        self.local = backend_factory()
        if filter != "native":  # the batched search's int8 filter copy (DeviceIndex.set_filter)
            self.local.set_filter(filter)
        self.merge = merge_fn
        self.n_rows = 0  # global rows [0, n_rows) hold data (the same value on every rank)
        self.coverage = RowCoverage()  # local rows of this rank's shard that hold data

    @property
    def written(self) -> int:
        """Local rows [0, written) of this rank's shard hold data, with no gap."""
        return self.coverage.prefix

    @property
    def n_local(self) -> int:
        """Rows of the global range [0, n_rows) this rank holds."""
        return (self.n_rows - self.rank + self.world - 1) // self.world if self.n_rows > self.rank else 0

    def owner(self, global_rows: torch.Tensor) -> torch.Tensor:
        return torch.remainder(global_rows, self.world)

    def upsert_rows(self, vecs: torch.Tensor, global_rows: torch.Tensor) -> int:
        """Called with the same (vecs, global_rows) on every rank; each rank writes the rows it owns."""
        gr = torch.as_tensor(global_rows, dtype=torch.int64).cpu()
        if gr.numel() == 0:
            return 0
        if int(gr.min()) < 0 or int(gr.max()) // self.world >= self.capacity:
            raise ValueError("row out of capacity")
        mine = self.owner(gr) == self.rank
        if bool(mine.any()):
            idx = torch.nonzero(mine).reshape(-1)
            loc = torch.div(gr[idx], self.world, rounding_mode="floor")
            self.local.upsert_rows(vecs[idx.to(vecs.device)], loc)
            self.coverage.add_rows(loc)
        self.n_rows = max(self.n_rows, int(gr.max()) + 1)
        return int(mine.sum())

    def upsert_local(self, vecs: torch.Tensor, local_rows: torch.Tensor) -> None:
        """Rank-local ingest (data-parallel embed → own shard, no collective): vecs go to this
        rank's local rows, i.e. global rows local * W + rank.  Rows are checked against the
        shard's capacity on the host (one small device→host read when they live on the GPU).
        Call ``publish_rows`` (or ``set_rows``) once every rank has ingested."""
        lr = torch.as_tensor(local_rows)
        if lr.numel() == 0:
            return
        lo, hi = (int(v) for v in torch.aminmax(lr.reshape(-1)))
        if lo < 0 or hi >= self.capacity:
            raise ValueError(f"local rows [{lo}, {hi}] outside the shard's capacity {self.capacity}")
        self.local.upsert_rows(vecs, lr)
        self.coverage.add_rows(lr)

    def _rows_ok(self, n_rows: int) -> bool:
        return (n_rows - self.rank + self.world - 1) // self.world <= self.written if n_rows > self.rank else True

    def set_rows(self, n_rows: int) -> None:
        """Publish the global row count (the same value on every rank).  Raises if this rank's
        part of [0, n_rows) reaches past its gap-free written prefix: unwritten slots are
        zero rows that would score 0 and come back as matches with ids that do not exist."""
        n_rows = int(n_rows)
        if n_rows < 0 or not self._rows_ok(n_rows):
            raise ValueError(f"rank {self.rank} has written {self.written} local rows: global rows [0, {n_rows}) "
                             f"need {(n_rows - self.rank + self.world - 1) // self.world}")
        self.n_rows = n_rows

    def publish_rows(self) -> int:
        """Collective: the largest global row count every rank's shard covers, from the ranks'
        written counts (rank r holds global rows r, r + W, ...: n_rows = min_r written_r·W + r),
        set on every rank and returned.  Ranks that ingested different counts stay consistent."""
        if self.world == 1:
            self.n_rows = self.written
            return self.n_rows
        dev = "cpu" if self.host_exchange else self.local.device
        t = torch.tensor([self.written], dtype=torch.int64, device=dev)
        allw = torch.empty((self.world,), dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(allw, t, group=self.group)
        self.n_rows = min(int(w) * self.world + r for r, w in enumerate(allw.cpu().tolist()))
        return self.n_rows

    def fill_random(self, seed: int, n_local: int) -> None:
        """Synthetic shard (benchmarks): every rank fills n_local rows, so the index holds
        n_local * W global rows."""
        self.local.fill_random(seed, 0, n_local)
        self.coverage.add(0, int(n_local))
        self.n_rows = n_local * self.world

    def search(self, queries: torch.Tensor, k: int, **kw):
        """Exact global top-k for the (replicated) queries: (scores [nq,k], global rows [nq,k]) on every rank.

        ``kw`` goes to the shard's search (e.g. ``mode="mfma"`` for the batched MFMA path)."""
        s, r = self.local.search(queries, k, self.n_local, **kw)
        if self.world == 1:
            return s, r
        nq = s.shape[0]
        dev = s.device
        if self.host_exchange:  # gloo: the exchange runs on host copies
            s, r = s.cpu(), r.cpu()
        gs = torch.empty((self.world * nq, k), dtype=s.dtype, device=s.device)
        gr = torch.empty((self.world * nq, k), dtype=r.dtype, device=r.device)
        dist.all_gather_into_tensor(gs, s.contiguous(), group=self.group)
        dist.all_gather_into_tensor(gr, r.contiguous(), group=self.group)
        gs, gr = gs.to(dev), gr.to(dev)
        return self.merge(gs.view(self.world, nq, k), gr.view(self.world, nq, k), k)

    # ---------------------------------------------------------- persistence --
    # Each rank snapshots its own shard (no collective): <path>/shard<rank>/
    # {rows.npy, norms.npy, manifest.json}; restore needs the same world size and
    # per-rank capacity, so global row numbers are unchanged.
    def save(self, path: str) -> None:
        import numpy as np

        d = os.path.join(path, f"shard{self.rank}")
        os.makedirs(d, exist_ok=True)
        rows, norms = self.local.export_rows(0, self.n_local)
        torch.cuda.synchronize()
        np.save(os.path.join(d, "rows.npy"), rows.cpu().numpy())
        np.save(os.path.join(d, "norms.npy"), norms.cpu().numpy())
        with open(os.path.join(d, "manifest.json"), "w") as f:
            json.dump({"format": 2, "rank": self.rank, "world": self.world, "dim": self.dim,
                       "routing": "round-robin", "capacity_per_rank": self.capacity, "n_rows": self.n_rows}, f)

    def load(self, path: str) -> None:
        import numpy as np

        d = os.path.join(path, f"shard{self.rank}")
        with open(os.path.join(d, "manifest.json")) as f:
            man = json.load(f)
        if man.get("format") != 2:
            raise ValueError(f"unsupported shard snapshot format {man.get('format')!r}")
        if (man["world"], man["capacity_per_rank"], man["dim"]) != (self.world, self.capacity, self.dim):
            raise ValueError("snapshot was taken with a different world size, capacity or dimension")
        rows = np.load(os.path.join(d, "rows.npy"), allow_pickle=False)
        norms = np.load(os.path.join(d, "norms.npy"), allow_pickle=False)
        self.n_rows = int(man["n_rows"])
        if self.n_local:
            self.local.import_rows(0, torch.from_numpy(rows), torch.from_numpy(norms))
        self.coverage = RowCoverage()
        self.coverage.add(0, self.n_local)

    def close(self) -> None:
        close = getattr(self.local, "close", None)
        if close:
            close()
