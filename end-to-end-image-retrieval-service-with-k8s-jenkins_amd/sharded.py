"""Row-sharded exact cosine index across the GPUs of one node (one process per GPU).

SURVEY §8(e): rows split contiguously — rank r owns global rows
[r*C, (r+1)*C) of a per-rank capacity C.  A query batch (identical on every
rank) is scanned by each rank's HIP kernel over its shard → local top-k
``(f32 score, i64 global row)``; one ``all_gather_into_tensor`` per output
(RCCL over xGMI; Q*k*12 B per rank) brings every rank's list to every rank, and
``rc_topk_merge`` merges them on the device with the same tie rule (score desc,
row asc).  Upserts need no collective: a row is written only by its owner.

Pinecone does the cross-partition merge server-side (the reference only sees
``index.query`` at ``retriever/utils.py:62``); this is the MI355X equivalent.
"""
from __future__ import annotations

import json
import os
from typing import Callable

import torch
import torch.distributed as dist


class ShardedIndex:
    def __init__(self, dim: int, dtype: str = "float16", capacity_per_rank: int = 1 << 20, group=None,
                 device=None, backend_factory: Callable | None = None, merge_fn: Callable | None = None):
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.dim = int(dim)
        self.capacity = int(capacity_per_rank)
        self.row_base = self.rank * self.capacity
        if backend_factory is None:
            from .index import DeviceIndex, topk_merge

            backend_factory = lambda: DeviceIndex(dim, dtype=dtype, capacity=capacity_per_rank, device=device,
                                                  row_base=self.row_base)
            merge_fn = merge_fn or topk_merge
        self.local = backend_factory()
        self.merge = merge_fn
        self.n_local = 0  # rows [0, n_local) of the shard hold data

    def owner(self, global_rows: torch.Tensor) -> torch.Tensor:
        return torch.div(global_rows, self.capacity, rounding_mode="floor")

    def upsert_rows(self, vecs: torch.Tensor, global_rows: torch.Tensor) -> int:
        """Called with the same (vecs, global_rows) on every rank; each rank writes the rows it owns."""
        mine = self.owner(global_rows.cpu()) == self.rank
        if bool(mine.any()):
            idx = torch.nonzero(mine).reshape(-1)
            local_rows = global_rows.cpu()[idx] - self.row_base
            self.local.upsert_rows(vecs[idx.to(vecs.device)], local_rows)
            self.n_local = max(self.n_local, int(local_rows.max()) + 1)
        return int(mine.sum())

    def fill_random(self, seed: int, n_local: int) -> None:
        self.local.fill_random(seed, 0, n_local)
        self.n_local = n_local

    def search(self, queries: torch.Tensor, k: int, **kw):
        """Exact global top-k for the (replicated) queries: (scores [nq,k], global rows [nq,k]) on every rank.

        ``kw`` goes to the shard's search (e.g. ``mode="mfma"`` for the batched MFMA path)."""
        s, r = self.local.search(queries, k, self.n_local, **kw)
        if self.world == 1:
            return s, r
        nq = s.shape[0]
        gs = torch.empty((self.world * nq, k), dtype=s.dtype, device=s.device)
        gr = torch.empty((self.world * nq, k), dtype=r.dtype, device=r.device)
        dist.all_gather_into_tensor(gs, s.contiguous(), group=self.group)
        dist.all_gather_into_tensor(gr, r.contiguous(), group=self.group)
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
            json.dump({"format": 1, "rank": self.rank, "world": self.world, "dim": self.dim,
                       "capacity_per_rank": self.capacity, "n_local": self.n_local}, f)

    def load(self, path: str) -> None:
        import numpy as np

        d = os.path.join(path, f"shard{self.rank}")
        with open(os.path.join(d, "manifest.json")) as f:
            man = json.load(f)
        if (man["world"], man["capacity_per_rank"], man["dim"]) != (self.world, self.capacity, self.dim):
            raise ValueError("snapshot was taken with a different world size, capacity or dimension")
        rows = np.load(os.path.join(d, "rows.npy"), allow_pickle=False)
        norms = np.load(os.path.join(d, "norms.npy"), allow_pickle=False)
        if man["n_local"]:
            self.local.import_rows(0, torch.from_numpy(rows), torch.from_numpy(norms))
        self.n_local = int(man["n_local"])

    def close(self) -> None:
        close = getattr(self.local, "close", None)
        if close:
            close()
