"""In-HBM exact cosine index behind Pinecone's ``Index`` shape.

Replaces the remote Pinecone index the reference opens in ``get_index``
(``ingesting/utils.py:23-38`` = ``retriever/utils.py:23-38``) and calls at
``index.upsert([(id, feature, metadata)])`` (``ingesting/main.py:156-158``),
``index.query(vector=..., top_k=..., include_values=True)["matches"]``
(``retriever/utils.py:62-64``) and ``index.fetch(ids=...)``
(``retriever/main.py:142``, consumed at ``:151-153``).

Split of work: string ids, metadata and the id → row map stay on the host
(Pinecone ids are uuid4 strings, ``ingesting/main.py:127``); the device holds
only the L2-normalised rows, written and searched by the HIP library through
the C ABI (``include/retrieval_core.h``).
"""
from __future__ import annotations

import json
import os
import threading
from typing import Any, Iterable, Sequence

import torch

from . import _lib
from ._lib import check, ptr, stream_ptr


def _device_index(device) -> int:
    if device is None:
        return torch.cuda.current_device()
    if isinstance(device, torch.device):
        return device.index if device.index is not None else torch.cuda.current_device()
    if isinstance(device, str):
        d = torch.device(device)
        return d.index if d.index is not None else torch.cuda.current_device()
    return int(device)


class DeviceIndex:
    """One ``rc_index`` handle: a contiguous block of row slots on one GPU (a shard)."""

    def __init__(self, dim: int, dtype: str = "float32", capacity: int = 1 << 20, device=None, row_base: int = 0):
        self.lib = _lib.load()
        if dtype not in _lib.DTYPES:
            raise ValueError(f"unknown index dtype {dtype!r}")
        self.dim = int(dim)
        self.dtype = dtype
        self.capacity = int(capacity)
        self.device_index = _device_index(device)
        self.device = torch.device("cuda", self.device_index)
        self.row_base = int(row_base)
        h = _lib.C.c_void_p()
        check(self.lib.rc_index_create(self.device_index, self.dim, _lib.DTYPES[dtype], self.capacity, self.row_base, _lib.C.byref(h)))
        self._h = h

    @property
    def handle(self):
        if self._h is None:
            raise RuntimeError("index is closed")
        return self._h

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            check(self.lib.rc_index_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def ld(self) -> int:
        ld = _lib.C.c_int64()
        check(self.lib.rc_index_info(self.handle, None, None, None, _lib.C.byref(ld)))
        return ld.value

    def reserve(self, max_nq: int, max_k: int) -> None:
        check(self.lib.rc_index_reserve(self.handle, int(max_nq), int(max_k)))

    def _vecs(self, vecs: torch.Tensor) -> torch.Tensor:
        if vecs.dim() == 1:
            vecs = vecs[None]
        if vecs.shape[-1] != self.dim:
            raise ValueError(f"Vector dimension {vecs.shape[-1]} does not match the dimension of the index {self.dim}")
        return vecs.to(device=self.device, dtype=torch.float32).contiguous()

    def upsert_rows(self, vecs: torch.Tensor, rows: torch.Tensor, stream=None) -> None:
        vecs = self._vecs(vecs)
        rows = rows.to(device=self.device, dtype=torch.int64).contiguous()
        if rows.numel() != vecs.shape[0]:
            raise ValueError("rows and vectors differ in length")
        check(self.lib.rc_index_upsert(self.handle, ptr(vecs), vecs.shape[0], ptr(rows), stream_ptr(stream)))

    def fetch_rows(self, rows: torch.Tensor, stream=None) -> torch.Tensor:
        rows = rows.to(device=self.device, dtype=torch.int64).contiguous()
        out = torch.empty((rows.numel(), self.dim), dtype=torch.float32, device=self.device)
        check(self.lib.rc_index_fetch(self.handle, ptr(rows), rows.numel(), ptr(out), stream_ptr(stream)))
        return out

    def search(self, queries: torch.Tensor, k: int, n_rows: int, stream=None, out=None, mode: str = "auto"):
        """Exact cosine top-k over rows [0, n_rows): (scores f32 [nq,k], global rows i64 [nq,k]).

        ``mode``: "scan" (HBM-bound streaming scan), "mfma" (batched filter GEMM +
        exact rescoring, f16/bf16 index) or "auto" (MFMA for >= 8 queries)."""
        if mode not in _lib.SEARCH_MODES:
            raise ValueError(f"unknown search mode {mode!r}")
        q = self._vecs(queries)
        nq = q.shape[0]
        if out is None:
            scores = torch.empty((nq, k), dtype=torch.float32, device=self.device)
            rows = torch.empty((nq, k), dtype=torch.int64, device=self.device)
        else:
            scores, rows = out
        check(self.lib.rc_index_search_ex(self.handle, ptr(q), nq, int(n_rows), int(k), ptr(scores), ptr(rows),
                                          _lib.SEARCH_MODES[mode], stream_ptr(stream)))
        return scores, rows

    def export_rows(self, row0: int, n: int, stream=None):
        """Raw stored rows [row0, row0+n) (storage dtype bits, ld-padded) and norms, on the device."""
        el = 4 if self.dtype in ("float32", "f32") else 2
        rows = torch.empty((n, self.ld * el), dtype=torch.uint8, device=self.device)
        norms = torch.empty((n,), dtype=torch.float32, device=self.device)
        check(self.lib.rc_index_export(self.handle, int(row0), int(n), ptr(rows), ptr(norms), stream_ptr(stream)))
        return rows, norms

    def import_rows(self, row0: int, rows: torch.Tensor, norms: torch.Tensor, stream=None) -> None:
        """Inverse of export_rows: write raw stored rows + norms at [row0, row0+n)."""
        el = 4 if self.dtype in ("float32", "f32") else 2
        rows = rows.to(device=self.device, dtype=torch.uint8).contiguous()
        norms = norms.to(device=self.device, dtype=torch.float32).contiguous()
        n = norms.numel()
        if rows.numel() != n * self.ld * el:
            raise ValueError("row bytes do not match the index layout (dimension / dtype)")
        check(self.lib.rc_index_import(self.handle, int(row0), n, ptr(rows), ptr(norms), stream_ptr(stream)))

    def fill_random(self, seed: int, row0: int, n: int, stream=None) -> None:
        check(self.lib.rc_index_fill_random(self.handle, int(seed), int(row0), int(n), stream_ptr(stream)))

    def stored_rows(self, rows: "torch.Tensor | int", stream=None) -> torch.Tensor:
        """The stored (normalised, dtype-rounded) rows as f32 — what search scores against."""
        if isinstance(rows, int):
            rows = torch.arange(rows, dtype=torch.int64)
        rows = rows.to(device=self.device, dtype=torch.int64).contiguous()
        out = torch.empty((rows.numel(), self.dim), dtype=torch.float32, device=self.device)
        check(self.lib.rc_index_fetch_stored(self.handle, ptr(rows), rows.numel(), ptr(out), stream_ptr(stream)))
        return out

    def timing(self, enable: bool) -> None:
        check(self.lib.rc_index_timing(self.handle, 1 if enable else 0))

    def timing_read(self):
        """Scan kernel: (total ms, launches, algorithmic bytes) since the last read."""
        ms = _lib.C.c_double()
        n = _lib.C.c_int64()
        b = _lib.C.c_double()
        check(self.lib.rc_index_timing_read(self.handle, _lib.C.byref(ms), _lib.C.byref(n), _lib.C.byref(b)))
        return ms.value, n.value, b.value

    def gemm_timing_read(self):
        """Batched filter GEMM: (total ms, launches, flops, fallback count) since the last read."""
        ms = _lib.C.c_double()
        n = _lib.C.c_int64()
        f = _lib.C.c_double()
        fb = _lib.C.c_int64()
        check(self.lib.rc_index_gemm_timing_read(self.handle, _lib.C.byref(ms), _lib.C.byref(n), _lib.C.byref(f),
                                                 _lib.C.byref(fb)))
        return ms.value, n.value, f.value, fb.value


def topk_merge(scores: torch.Tensor, rows: torch.Tensor, k: int, stream=None):
    """Merge [nlists, nq, k_in] sorted candidate lists into [nq, k] on the device (rc_topk_merge)."""
    lib = _lib.load()
    scores = scores.contiguous()
    rows = rows.contiguous()
    nlists, nq, k_in = scores.shape
    out_s = torch.empty((nq, k), dtype=torch.float32, device=scores.device)
    out_r = torch.empty((nq, k), dtype=torch.int64, device=scores.device)
    check(lib.rc_topk_merge(ptr(scores), ptr(rows), nlists, nq, k_in, k, ptr(out_s), ptr(out_r), stream_ptr(stream)))
    return out_s, out_r


def _as_vector(values: Any, dim: int) -> list[float]:
    if isinstance(values, torch.Tensor):
        values = values.detach().cpu().reshape(-1).tolist()
    vals = [float(v) for v in values]
    if len(vals) != dim:
        raise ValueError(f"Vector dimension {len(vals)} does not match the dimension of the index {dim}")
    if not any(v != 0.0 for v in vals):
        raise ValueError("Dense vectors must contain at least one non-zero value for the cosine metric")
    return vals


class Index:
    """Pinecone-shaped index (what ``get_index`` returns), cosine metric only.

    ``upsert(vectors)`` accepts ``(id, values)``, ``(id, values, metadata)``
    tuples or ``{"id", "values", "metadata"}`` dicts and overwrites existing
    ids; ``query`` returns ``{"matches": [{"id", "score", ["values"],
    ["metadata"]}], "namespace": ""}`` best first; ``fetch`` returns
    ``{"vectors": {id: {"id", "values", "metadata"}}, "namespace": ""}``.
    """

    def __init__(self, name: str, dimension: int = 768, metric: str = "cosine", dtype: str = "float32",
                 capacity: int = 1 << 20, device=None):
        if metric != "cosine":
            raise ValueError("only metric='cosine' is supported")
        self.name = name
        self.dimension = int(dimension)
        self.metric = metric
        self._dev = DeviceIndex(self.dimension, dtype=dtype, capacity=capacity, device=device)
        self._rows: dict[str, int] = {}
        self._ids: list[str] = []
        self._meta: dict[str, dict] = {}
        self._mu = threading.Lock()

    @property
    def device_index(self) -> DeviceIndex:
        return self._dev

    def __len__(self) -> int:
        return len(self._ids)

    def _normalize_items(self, vectors: Iterable) -> list[tuple[str, list[float], dict]]:
        items = []
        for v in vectors:
            if isinstance(v, dict):
                vid, vals, md = v["id"], v["values"], v.get("metadata") or {}
            else:
                v = tuple(v)
                if len(v) == 2:
                    (vid, vals), md = v, {}
                elif len(v) == 3:
                    vid, vals, md = v
                    md = md or {}
                else:
                    raise ValueError("vectors must be (id, values[, metadata]) tuples or dicts")
            if not isinstance(vid, str) or not vid:
                raise ValueError("vector id must be a non-empty string")
            items.append((vid, _as_vector(vals, self.dimension), dict(md)))
        return items

    def upsert(self, vectors: Sequence, namespace: str = "") -> dict:
        items = self._normalize_items(vectors)
        if not items:
            return {"upserted_count": 0}
        with self._mu:
            rows = []
            for vid, _, md in items:
                r = self._rows.get(vid)
                if r is None:
                    r = len(self._ids)
                    if r >= self._dev.capacity:
                        raise ValueError(f"index {self.name!r} is full ({self._dev.capacity} vectors)")
                    self._rows[vid] = r
                    self._ids.append(vid)
                rows.append(r)
                self._meta[vid] = md
            vecs = torch.tensor([it[1] for it in items], dtype=torch.float32).to(self._dev.device)
            rows_t = torch.tensor(rows, dtype=torch.int64).to(self._dev.device)
            self._dev.upsert_rows(vecs, rows_t)
            torch.cuda.current_stream(self._dev.device).synchronize()
        return {"upserted_count": len(items)}

    def query(self, vector=None, top_k: int = 10, include_values: bool = False, include_metadata: bool = False,
              id: str | None = None, namespace: str = "", **_: Any) -> dict:
        if vector is None and id is None:
            raise ValueError("query needs a vector or an id")
        if top_k < 1:
            raise ValueError("top_k must be a positive integer")
        with self._mu:
            if vector is None:
                vec = self.fetch([id])["vectors"].get(id)
                if vec is None:
                    return {"matches": [], "namespace": namespace}
                vector = vec["values"]
            q = torch.tensor([_as_vector(vector, self.dimension)], dtype=torch.float32).to(self._dev.device)
            n = len(self._ids)
            k = min(int(top_k), _lib.RC_TOPK_MAX)
            matches = []
            if n > 0:
                scores, rows = self._dev.search(q, k, n)
                scores = scores[0].cpu().tolist()
                rows = rows[0].cpu().tolist()
                sel = [(s, r) for s, r in zip(scores, rows) if r >= 0]
                vals = None
                if include_values and sel:
                    vals = self._dev.fetch_rows(torch.tensor([r for _, r in sel], dtype=torch.int64)).cpu().tolist()
                for j, (s, r) in enumerate(sel):
                    m = {"id": self._ids[r], "score": float(s)}
                    if include_values:
                        m["values"] = vals[j]
                    if include_metadata:
                        m["metadata"] = dict(self._meta.get(self._ids[r], {}))
                    matches.append(m)
        return {"matches": matches, "namespace": namespace}

    def fetch(self, ids: Sequence[str], namespace: str = "") -> dict:
        found = [(i, self._rows[i]) for i in ids if i in self._rows]
        vectors = {}
        if found:
            vals = self._dev.fetch_rows(torch.tensor([r for _, r in found], dtype=torch.int64)).cpu().tolist()
            for (vid, _), v in zip(found, vals):
                vectors[vid] = {"id": vid, "values": v, "metadata": dict(self._meta.get(vid, {}))}
        return {"vectors": vectors, "namespace": namespace}

    # ---------------------------------------------------------- persistence --
    # Pinecone keeps an index durable server-side (the reference only opens it by
    # name, ingesting/utils.py:23-38); the in-HBM index is saved to a directory:
    # manifest.json (name, dimension, dtype, ids in row order, metadata) +
    # rows.npy (raw stored bytes, exactly what search scores) + norms.npy.
    SNAPSHOT_FORMAT = 1

    def save(self, path: str) -> None:
        with self._mu:
            os.makedirs(path, exist_ok=True)
            n = len(self._ids)
            rows, norms = self._dev.export_rows(0, n)
            torch.cuda.current_stream(self._dev.device).synchronize()
            import numpy as np

            np.save(os.path.join(path, "rows.npy"), rows.cpu().numpy())
            np.save(os.path.join(path, "norms.npy"), norms.cpu().numpy())
            manifest = {"format": self.SNAPSHOT_FORMAT, "name": self.name, "dimension": self.dimension,
                        "metric": self.metric, "dtype": self._dev.dtype, "ld": self._dev.ld, "count": n,
                        "capacity": self._dev.capacity,
                        "ids": list(self._ids), "metadata": {i: self._meta.get(i, {}) for i in self._ids}}
            tmp = os.path.join(path, "manifest.json.tmp")
            with open(tmp, "w") as f:
                json.dump(manifest, f)
            os.replace(tmp, os.path.join(path, "manifest.json"))  # the manifest lands last

    @classmethod
    def load(cls, path: str, capacity: int | None = None, device=None) -> "Index":
        import numpy as np

        with open(os.path.join(path, "manifest.json")) as f:
            man = json.load(f)
        if man.get("format") != cls.SNAPSHOT_FORMAT:
            raise ValueError(f"unsupported snapshot format {man.get('format')!r}")
        n = int(man["count"])
        idx = cls(man["name"], dimension=man["dimension"], metric=man["metric"], dtype=man["dtype"],
                  capacity=max(int(capacity or man.get("capacity", 0)), n, 1), device=device)
        if idx._dev.ld != man["ld"]:
            raise ValueError("snapshot row layout does not match this build")
        rows = np.load(os.path.join(path, "rows.npy"), allow_pickle=False)
        norms = np.load(os.path.join(path, "norms.npy"), allow_pickle=False)
        if rows.shape[0] != n or norms.shape[0] != n or len(man["ids"]) != n:
            raise ValueError("snapshot files disagree on the vector count")
        if n:
            idx._dev.import_rows(0, torch.from_numpy(rows), torch.from_numpy(norms))
            torch.cuda.current_stream(idx._dev.device).synchronize()
        idx._ids = list(man["ids"])
        idx._rows = {vid: r for r, vid in enumerate(idx._ids)}
        idx._meta = {vid: dict(man["metadata"].get(vid, {})) for vid in idx._ids}
        return idx

    def describe_index_stats(self) -> dict:
        return {"dimension": self.dimension, "index_fullness": len(self._ids) / self._dev.capacity,
                "total_vector_count": len(self._ids), "namespaces": {"": {"vector_count": len(self._ids)}}}
