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

import array
import json
import os
import threading
from typing import Any, Iterable, Sequence

import numpy as np
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
    """One ``rc_index`` handle: a block of row slots on one GPU (a shard).

    A search returns ``row_base + local_row * row_stride`` (``set_row_map``):
    the global rows of a round-robin shard."""

    def __init__(self, dim: int, dtype: str = "float32", capacity: int = 1 << 20, device=None, row_base: int = 0,
                 row_stride: int = 1, _handle=None):
        self.lib = _lib.load()
        if dtype not in _lib.DTYPES:
            raise ValueError(f"unknown index dtype {dtype!r}")
        self.dim = int(dim)
        self.dtype = dtype
        self.device_index = _device_index(device)
        self.device = torch.device("cuda", self.device_index)
        self.row_base = int(row_base)
        self.row_stride = int(row_stride)
        self._owned = _handle is None
        if _handle is None:
            h = _lib.C.c_void_p()
            check(self.lib.rc_index_create(self.device_index, self.dim, _lib.DTYPES[dtype], int(capacity), self.row_base,
                                           _lib.C.byref(h)))
            self._h = h
            if self.row_stride != 1:
                self.set_row_map(self.row_base, self.row_stride)
        else:  # a shard borrowed from an rc_sharded handle (owned there)
            self._h = _handle

    @property
    def handle(self):
        if self._h is None:
            raise RuntimeError("index is closed")
        return self._h

    @property
    def capacity(self) -> int:
        cap = _lib.C.c_int64()
        check(self.lib.rc_index_info(self.handle, None, None, _lib.C.byref(cap), None))
        return cap.value

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            if self._owned:
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

    def set_row_map(self, row_base: int, row_stride: int = 1) -> None:
        check(self.lib.rc_index_set_row_map(self.handle, int(row_base), int(row_stride)))
        self.row_base, self.row_stride = int(row_base), int(row_stride)

    def grow(self, new_capacity: int, stream=None) -> None:
        check(self.lib.rc_index_grow(self.handle, int(new_capacity), stream_ptr(stream)))

    def reserve(self, max_nq: int, max_k: int) -> None:
        check(self.lib.rc_index_reserve(self.handle, int(max_nq), int(max_k)))

    def set_filter(self, kind: str, stream=None) -> None:
        """Filter copy of the batched search (rc_index_set_filter): "native" (the filter GEMM
        reads the stored rows) or "i8" (an int8 copy of every row, int8 MFMA at twice the f16
        rate; results unchanged — candidates are rescored exactly on the stored rows)."""
        if kind not in _lib.FILTERS:
            raise ValueError(f"unknown filter {kind!r} (expected one of {sorted(_lib.FILTERS)})")
        check(self.lib.rc_index_set_filter(self.handle, _lib.FILTERS[kind], stream_ptr(stream)))

    @property
    def filter(self) -> str:
        k = _lib.C.c_int()
        check(self.lib.rc_index_get_filter(self.handle, _lib.C.byref(k)))
        return {v: n for n, v in _lib.FILTERS.items()}[k.value]

    def _vecs(self, vecs: torch.Tensor) -> torch.Tensor:
        if vecs.dim() == 1:
            vecs = vecs[None]
        if vecs.shape[-1] != self.dim:
            raise ValueError(f"Vector dimension {vecs.shape[-1]} does not match the dimension of the index {self.dim}")
        return vecs.to(device=self.device, dtype=torch.float32).contiguous()

    def upsert_rows(self, vecs: torch.Tensor, rows: torch.Tensor, stream=None) -> None:
        """rows must be distinct (rc_index_upsert); callers with repeated ids dedupe first."""
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


class Record(dict):
    """A query match or fetched vector in Pinecone's shape (``{"id", "score" | "values",
    "metadata"}``) whose ``"values"`` entry stays a float32 row until something reads it.

    The reference's ``search`` asks for ``include_values=True`` and keeps only the ids
    (``retriever/utils.py:62-65``), so building 5 x 768 Python floats per request is work no
    caller of that path sees.  Every read path of the dict — ``[]``, ``get``, ``items``,
    ``values``, iteration with ``dict(...)`` / ``{**m}``, ``==``, ``copy``, ``repr``, pickling,
    ``json.dumps`` (which calls ``items()`` on a dict subclass), ``|`` — first turns the row into
    the list of Python floats a plain dict would hold, once; writing or deleting ``"values"``
    drops the pending row, and ``update`` / ``|=`` load it first."""

    __slots__ = ("_row",)

    def __init__(self, row: np.ndarray | None = None, **fields):
        super().__init__(fields)
        self._row = row
        if row is not None:
            dict.__setitem__(self, "values", None)

    def _load(self) -> None:
        row = self._row
        if row is not None:
            self._row = None
            dict.__setitem__(self, "values", row.astype(np.float64).tolist())

    def __getitem__(self, key):
        if key == "values":
            self._load()
        return dict.__getitem__(self, key)

    def get(self, key, default=None):
        if key == "values":
            self._load()
        return dict.get(self, key, default)

    def __iter__(self):  # a Python-level __iter__ sends dict(m) / {**m} through keys() + __getitem__
        return dict.__iter__(self)

    def items(self):
        self._load()
        return dict.items(self)

    def values(self):
        self._load()
        return dict.values(self)

    def copy(self):
        self._load()
        return dict(dict.items(self))

    def pop(self, key, *default):
        self._load()
        return dict.pop(self, key, *default)

    def popitem(self):
        self._load()
        return dict.popitem(self)

    def setdefault(self, key, default=None):
        self._load()
        return dict.setdefault(self, key, default)

    # writes: a new "values" (or its removal) supersedes the pending row, so the row must not
    # come back on the next read; any other key leaves it pending
    def __setitem__(self, key, value):
        if key == "values":
            self._row = None
        dict.__setitem__(self, key, value)

    def __delitem__(self, key):
        if key == "values":
            self._row = None
        dict.__delitem__(self, key)

    def update(self, *a, **kw):
        self._load()
        dict.update(self, *a, **kw)

    def __or__(self, other):
        self._load()
        return dict(dict.items(self)) | dict(other)

    def __ror__(self, other):
        self._load()
        return dict(other) | dict(dict.items(self))

    def __ior__(self, other):
        self.update(other)
        return self

    def __eq__(self, other):
        self._load()
        if isinstance(other, Record):
            other._load()
        return dict.__eq__(self, other)

    def __ne__(self, other):
        return not self.__eq__(other)

    __hash__ = None

    def __repr__(self):
        self._load()
        return dict.__repr__(self)

    def __reduce__(self):
        self._load()
        return (dict, (dict(dict.items(self)),))


class F32List(list):
    """A list of floats (an embedding as ``/embed`` returns it) that also carries the float32
    array it was made from, so an in-process ``search`` (retriever/main.py:122-128: the
    feature goes straight back into ``index.query``) skips re-parsing 768 Python floats.  Any
    mutation drops the array; the list is then parsed like any other."""

    __slots__ = ("f32",)

    def __init__(self, values=(), f32: np.ndarray | None = None):
        super().__init__(values)
        self.f32 = f32

    def __setitem__(self, *a):
        self.f32 = None
        return list.__setitem__(self, *a)

    def __delitem__(self, *a):
        self.f32 = None
        return list.__delitem__(self, *a)

    def __iadd__(self, other):
        self.f32 = None
        return list.__iadd__(self, other)

    def __imul__(self, n):
        self.f32 = None
        return list.__imul__(self, n)

    def __reduce__(self):  # pickles / copies as the plain list
        return (list, (list(self),))


def _invalidating(name):
    base = getattr(list, name)

    def method(self, *a, **k):
        self.f32 = None
        return base(self, *a, **k)

    method.__name__ = name
    return method


for _m in ("append", "extend", "insert", "pop", "remove", "reverse", "sort", "clear"):
    setattr(F32List, _m, _invalidating(_m))
del _m


def _as_vector(values: Any, dim: int) -> list[float]:
    if isinstance(values, torch.Tensor):
        values = values.detach().cpu().reshape(-1).tolist()
    vals = [float(v) for v in values]
    if len(vals) != dim:
        raise ValueError(f"Vector dimension {len(vals)} does not match the dimension of the index {dim}")
    if not any(v != 0.0 for v in vals):
        raise ValueError("Dense vectors must contain at least one non-zero value for the cosine metric")
    return vals


def _as_vector_np(values: Any, dim: int) -> np.ndarray:
    """``_as_vector`` as a C-contiguous f32 [1, dim] host array (the request path: no per-element
    Python loop)."""
    if type(values) is F32List and values.f32 is not None:  # an in-process embedding: its own f32 row
        a = values.f32
    elif isinstance(values, torch.Tensor):
        a = values.detach().to(device="cpu", dtype=torch.float32).reshape(-1).numpy()
    else:
        a = None
        if isinstance(values, (list, tuple)):
            try:  # a JSON list of floats: array('f') converts it ~4x faster than np.asarray (same f32 rounding)
                a = np.frombuffer(array.array("f", values), dtype=np.float32)
            except TypeError:
                pass
        if a is None:
            a = np.asarray(values, dtype=np.float32)
            if a.ndim != 1:  # as _as_vector: float() of a nested element raises, nothing is flattened
                raise TypeError(f"a query vector must be a flat sequence of numbers (got shape {a.shape})")
    if a.shape[0] != dim:
        raise ValueError(f"Vector dimension {a.shape[0]} does not match the dimension of the index {dim}")
    if not a.any():
        raise ValueError("Dense vectors must contain at least one non-zero value for the cosine metric")
    return np.ascontiguousarray(a[None])


class ShardSet:
    """One ``rc_sharded`` handle: ``n`` shards (``rc_index`` each) in this process.

    Global row g lives on shard ``g % n`` as local row ``g // n`` (round-robin,
    SURVEY §8(e)); ``devices[s]`` is shard s's GPU (entries may repeat), and
    ``devices[0]`` (the leader) holds queries and merged results."""

    def __init__(self, dim: int, dtype: str = "float32", capacity_per_shard: int = 1 << 20, devices=None):
        self.lib = _lib.load()
        if dtype not in _lib.DTYPES:
            raise ValueError(f"unknown index dtype {dtype!r}")
        devs = [_device_index(d) for d in (devices if devices is not None else [None])]
        if not devs:
            raise ValueError("a sharded index needs at least one device")
        self.dim = int(dim)
        self.dtype = dtype
        self.devices = devs
        self.n = len(devs)
        self.device = torch.device("cuda", devs[0])
        arr = (_lib.C.c_int * self.n)(*devs)
        h = _lib.C.c_void_p()
        check(self.lib.rc_sharded_create(self.n, arr, self.dim, _lib.DTYPES[dtype], int(capacity_per_shard),
                                         _lib.C.byref(h)))
        self._h = h
        # rows upsert_parts had to copy from another GPU than their shard's (an EmbedderPool
        # batch whose planned rows shifted under a concurrent ingest): results stay exact,
        # this counts the extra xGMI traffic
        self.cross_device_rows = 0
        self._qbufs: dict = {}  # query_host's reused host buffers per (nq, k, values)
        self._query_fn = self.lib.rc_sharded_query_host
        self._shards = []
        for sh in range(self.n):
            ih = _lib.C.c_void_p()
            check(self.lib.rc_sharded_shard(h, sh, _lib.C.byref(ih)))
            self._shards.append(DeviceIndex(dim, dtype=dtype, device=devs[sh], row_base=sh, row_stride=self.n, _handle=ih))

    @property
    def handle(self):
        if self._h is None:
            raise RuntimeError("index is closed")
        return self._h

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            for d in self._shards:
                d.close()
            check(self.lib.rc_sharded_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def capacity_per_shard(self) -> int:
        cap = _lib.C.c_int64()
        check(self.lib.rc_sharded_info(self.handle, None, _lib.C.byref(cap), None))
        return cap.value

    @property
    def capacity(self) -> int:
        return self.capacity_per_shard * self.n

    @property
    def ld(self) -> int:
        ld = _lib.C.c_int64()
        check(self.lib.rc_sharded_info(self.handle, None, None, _lib.C.byref(ld)))
        return ld.value

    def force_remote(self) -> None:
        """Test hook (rc_sharded_force_remote): every shard but the leader through the
        cross-device path, as on a multi-GPU node, even when the shards share one GPU."""
        check(self.lib.rc_sharded_force_remote(self.handle))

    def shard(self, s: int) -> DeviceIndex:
        return self._shards[s]

    def shard_rows(self, s: int, n_rows: int) -> int:
        """How many of the global rows [0, n_rows) shard s holds."""
        return (n_rows - s + self.n - 1) // self.n if n_rows > s else 0

    def grow(self, new_capacity_per_shard: int) -> None:
        check(self.lib.rc_sharded_grow(self.handle, int(new_capacity_per_shard)))

    def set_filter(self, kind: str) -> None:
        """``DeviceIndex.set_filter`` on every shard."""
        if kind not in _lib.FILTERS:
            raise ValueError(f"unknown filter {kind!r} (expected one of {sorted(_lib.FILTERS)})")
        check(self.lib.rc_sharded_set_filter(self.handle, _lib.FILTERS[kind]))

    @property
    def filter(self) -> str:
        return self._shards[0].filter

    def upsert_rows(self, vecs: torch.Tensor, rows) -> None:
        """vecs f32 [n, dim] (any device; moved to the leader), rows: global rows (host)."""
        if vecs.dim() == 1:
            vecs = vecs[None]
        if vecs.shape[-1] != self.dim:
            raise ValueError(f"Vector dimension {vecs.shape[-1]} does not match the dimension of the index {self.dim}")
        vecs = vecs.to(device=self.device, dtype=torch.float32).contiguous()
        rows = torch.as_tensor(rows, dtype=torch.int64).cpu().contiguous()
        if rows.numel() != vecs.shape[0]:
            raise ValueError("rows and vectors differ in length")
        check(self.lib.rc_sharded_upsert(self.handle, ptr(vecs), vecs.shape[0], ptr(rows), stream_ptr(None)))

    def upsert_parts(self, parts) -> None:
        """Upsert vectors that already live on several devices (an ``EmbedderPool`` batch):
        ``parts`` = [(global rows: host i64 [m], vecs: f32 [m, dim] on any GPU)].  Each part's
        rows go straight to their shards: a shard on the part's own device takes its subset
        in place (no copy at all when the pool member and the shard share the GPU, the
        common case), any other shard gets only its subset copied over.  Synchronous per
        shard device, like ``upsert_rows``."""
        touched = set()
        for rows, vecs in parts:
            rows = torch.as_tensor(rows, dtype=torch.int64).cpu().reshape(-1)
            if rows.numel() == 0:
                continue
            if vecs.dim() != 2 or vecs.shape[0] != rows.numel() or vecs.shape[1] != self.dim:
                raise ValueError("each part needs vecs [len(rows), dim]")
            if int(rows.min()) < 0 or int(rows.max()) // self.n >= self.capacity_per_shard:
                raise ValueError("row out of capacity")
            sh = torch.remainder(rows, self.n)
            for s in torch.unique(sh).tolist():
                sel = torch.nonzero(sh == s).reshape(-1)
                d = self.devices[s]
                if vecs.device != torch.device("cuda", d):
                    self.cross_device_rows += int(sel.numel())
                v = vecs if sel.numel() == rows.numel() else vecs[sel.to(vecs.device)]
                with torch.cuda.device(d):
                    v = v.to(device=torch.device("cuda", d), dtype=torch.float32).contiguous()
                    self._shards[s].upsert_rows(v, torch.div(rows[sel], self.n, rounding_mode="floor"))
                touched.add(d)
        for d in touched:
            torch.cuda.synchronize(d)

    def query_host(self, q: np.ndarray, k: int, n_rows: int, with_values: bool):
        """Host f32 [nq, dim] → host (scores [nq, k], global rows [nq, k], values [nq, k, dim] or
        None): rc_sharded_query_host — one H2D copy, the search and the matched rows' gather, one
        D2H copy, one synchronisation.  The arrays are this ShardSet's reused buffers: valid
        until its next query_host call (the Index consumes them under its lock)."""
        nq = int(q.shape[0])
        key = (nq, int(k), bool(with_values))
        bufs = self._qbufs.get(key)
        if bufs is None:
            if len(self._qbufs) > 16:
                self._qbufs.clear()
            sc = np.empty((nq, k), np.float32)
            rw = np.empty((nq, k), np.int64)
            val = np.empty((nq, k, self.dim), np.float32) if with_values else None
            # the buffers' addresses once (ctypes attribute reads cost ~1 us each per call)
            ptrs = (int(bool(with_values)), sc.ctypes.data, rw.ctypes.data, val.ctypes.data if val is not None else None)
            bufs = (sc, rw, val, ptrs)
            self._qbufs[key] = bufs
        sc, rw, val, ptrs = bufs
        h = self._h
        if h is None:
            raise RuntimeError("index is closed")
        check(self._query_fn(h, q.ctypes.data, nq, n_rows, k, ptrs[0], ptrs[1], ptrs[2], ptrs[3]))
        return sc, rw, val

    def fetch_rows(self, rows, stored: bool = False) -> torch.Tensor:
        """Host f32 [n, dim]: the upserted values (or, ``stored``, the normalised stored rows)."""
        rows = torch.as_tensor(rows, dtype=torch.int64).cpu().contiguous()
        out = torch.empty((rows.numel(), self.dim), dtype=torch.float32)
        if rows.numel():
            check(self.lib.rc_sharded_fetch(self.handle, ptr(rows), rows.numel(), ptr(out), 1 if stored else 0))
        return out

    def search(self, queries: torch.Tensor, k: int, n_rows: int, mode: str = "auto", stream=None):
        """Exact cosine top-k over global rows [0, n_rows): (scores f32 [nq,k], rows i64 [nq,k]) on the leader."""
        if mode not in _lib.SEARCH_MODES:
            raise ValueError(f"unknown search mode {mode!r}")
        if queries.dim() == 1:
            queries = queries[None]
        q = queries.to(device=self.device, dtype=torch.float32).contiguous()
        nq = q.shape[0]
        scores = torch.empty((nq, k), dtype=torch.float32, device=self.device)
        rows = torch.empty((nq, k), dtype=torch.int64, device=self.device)
        check(self.lib.rc_sharded_search(self.handle, ptr(q), nq, int(n_rows), int(k), ptr(scores), ptr(rows),
                                         _lib.SEARCH_MODES[mode], stream_ptr(stream)))
        return scores, rows

    # raw stored rows in GLOBAL row order (the snapshot layout, independent of the shard count)
    def export_rows(self, n_rows: int):
        import numpy as np

        el = 4 if self.dtype in ("float32", "f32") else 2
        rows = np.zeros((n_rows, self.ld * el), dtype=np.uint8)
        norms = np.zeros((n_rows,), dtype=np.float32)
        for s in range(self.n):
            m = self.shard_rows(s, n_rows)
            if m == 0:
                continue
            r, nr = self._shards[s].export_rows(0, m)
            torch.cuda.synchronize(self._shards[s].device)
            rows[s::self.n] = r.cpu().numpy()
            norms[s::self.n] = nr.cpu().numpy()
        return rows, norms

    def import_rows(self, rows, norms) -> None:
        n_rows = len(norms)
        for s in range(self.n):
            if self.shard_rows(s, n_rows) == 0:
                continue
            self._shards[s].import_rows(0, torch.from_numpy(rows[s::self.n].copy()),
                                        torch.from_numpy(norms[s::self.n].copy()))
            torch.cuda.synchronize(self._shards[s].device)


class Index:
    """Pinecone-shaped index (what ``get_index`` returns), cosine metric only.

    ``upsert(vectors)`` accepts ``(id, values)``, ``(id, values, metadata)``
    tuples or ``{"id", "values", "metadata"}`` dicts and overwrites existing
    ids (within one call the last occurrence of an id wins); ``query`` returns
    ``{"matches": [{"id", "score", ["values"], ["metadata"]}], "namespace": ""}``
    best first; ``fetch`` returns ``{"vectors": {id: {"id", "values",
    "metadata"}}, "namespace": ""}``.

    The rows live on ``shards`` shards (``devices``: one GPU per shard, entries
    may repeat; default one shard on ``device``), routed round-robin by the
    row number the host assigns each new id, and searched as ONE exact index
    (``rc_sharded``): results are identical to a single-shard index holding the
    same vectors.  Capacity grows on demand (doubling), as a Pinecone index
    has no fixed size.
    """

    def __init__(self, name: str, dimension: int = 768, metric: str = "cosine", dtype: str = "float32",
                 capacity: int = 1 << 20, device=None, shards: int | None = None, devices=None,
                 filter: str = "native"):
        if metric != "cosine":
            raise ValueError("only metric='cosine' is supported")
        if filter not in _lib.FILTERS:
            raise ValueError(f"unknown filter {filter!r} (expected one of {sorted(_lib.FILTERS)})")
        if devices is None:
            devices = [device] * int(shards or 1)
        self.name = name
        self.dimension = int(dimension)
        self.metric = metric
        n = len(devices)
        self._set = ShardSet(self.dimension, dtype=dtype, capacity_per_shard=max(1, -(-int(capacity) // n)),
                             devices=devices)
        if filter != "native":
            self._set.set_filter(filter)
        self._rows: dict[str, int] = {}
        self._ids: list[str] = []
        self._meta: dict[str, dict] = {}
        self._mu = threading.Lock()
        # values the last query(include_values=True) fetched, valid until the next upsert: the
        # reference's search (retriever/utils.py:62-64) asks for values and its caller then
        # fetches the same ids (retriever/main.py:142) — each row leaves the GPU once
        self._gen = 0
        self._recent: tuple[int, dict[str, np.ndarray]] = (-1, {})

    @property
    def shard_set(self) -> ShardSet:
        return self._set

    @property
    def dtype(self) -> str:
        return self._set.dtype

    @property
    def capacity(self) -> int:
        return self._set.capacity

    @property
    def shard_devices(self) -> list[int]:
        """GPU of each shard (global row g lives on shard g % len(shard_devices))."""
        return list(self._set.devices)

    def __len__(self) -> int:
        return len(self._ids)

    def close(self) -> None:
        self._set.close()

    def _normalize_items(self, vectors: Iterable) -> list[tuple[str, list[float], dict]]:
        items: dict[str, tuple[str, list[float], dict]] = {}
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
            # one row per id: a repeated id in one call keeps its LAST values (two
            # writes of one row slot in the same launch would interleave)
            items[vid] = (vid, _as_vector(vals, self.dimension), dict(md))
        return list(items.values())

    def _ensure_capacity(self, n_total: int) -> None:
        if n_total <= self._set.capacity:
            return
        per = self._set.capacity_per_shard
        need = -(-n_total // self._set.n)
        while per < need:
            per *= 2
        self._set.grow(per)

    def upsert(self, vectors: Sequence, namespace: str = "") -> dict:
        items = self._normalize_items(vectors)
        if not items:
            return {"upserted_count": 0}
        vecs = torch.tensor([it[1] for it in items], dtype=torch.float32)
        with self._mu:
            self._upsert_locked(items, vecs)
        return {"upserted_count": len(items)}

    def upsert_tensor(self, ids: Sequence[str], vecs, metadata: Sequence[dict] | None = None) -> dict:
        """Batched upsert of device-resident vectors (the ingest path: embeddings never leave HBM).

        ``vecs``: f32 [len(ids), dimension] on a GPU, or a list of parts ``(positions,
        tensor)`` — the vectors of ``ids[positions]`` on whatever GPU produced them (an
        ``EmbedderPool`` batch): each goes straight to its shard's GPU.  Same semantics as
        ``upsert`` (overwrite by id, last occurrence wins)."""
        if isinstance(vecs, (list, tuple)):
            return self._upsert_parts(ids, vecs, metadata)
        if vecs.dim() != 2 or vecs.shape[0] != len(ids) or vecs.shape[1] != self.dimension:
            raise ValueError("vecs must be [len(ids), dimension]")
        metadata = list(metadata) if metadata is not None else [{}] * len(ids)
        if len(metadata) != len(ids):
            raise ValueError("metadata and ids differ in length")
        last: dict[str, int] = {}
        for i, vid in enumerate(ids):
            if not isinstance(vid, str) or not vid:
                raise ValueError("vector id must be a non-empty string")
            last[vid] = i
        keep = list(last.values())
        if len(keep) != len(ids):
            vecs = vecs[torch.tensor(keep, dtype=torch.int64, device=vecs.device)]
        nonzero = (vecs != 0).any(dim=1).all()  # queued behind the producer of vecs; read below
        items = [(ids[i], None, dict(metadata[i] or {})) for i in keep]
        if not bool(nonzero):
            raise ValueError("Dense vectors must contain at least one non-zero value for the cosine metric")
        with self._mu:
            self._upsert_locked(items, vecs)
        return {"upserted_count": len(items)}

    def _upsert_parts(self, ids, parts, metadata) -> dict:
        metadata = list(metadata) if metadata is not None else [{}] * len(ids)
        if len(metadata) != len(ids):
            raise ValueError("metadata and ids differ in length")
        where: dict[int, tuple[int, int]] = {}  # position -> (part, offset)
        for pi, (pos, t) in enumerate(parts):
            pos = [int(p) for p in pos]
            if t.dim() != 2 or t.shape[0] != len(pos) or t.shape[1] != self.dimension:
                raise ValueError("each part needs vectors [len(positions), dimension]")
            for o, p in enumerate(pos):
                where[p] = (pi, o)
        if sorted(where) != list(range(len(ids))):
            raise ValueError("the parts must cover every position of ids exactly once")
        last: dict[str, int] = {}
        for i, vid in enumerate(ids):
            if not isinstance(vid, str) or not vid:
                raise ValueError("vector id must be a non-empty string")
            last[vid] = i
        keep = list(last.values())
        for _, t in parts:
            if t.shape[0] and not bool((t != 0).any(dim=1).all()):
                raise ValueError("Dense vectors must contain at least one non-zero value for the cosine metric")
        items = [(ids[i], None, dict(metadata[i] or {})) for i in keep]
        with self._mu:
            rows = self._plan_rows(items)
            sel = [[] for _ in parts]  # per part: (offset, global row) of the kept positions
            for i, r in zip(keep, rows):
                pi, o = where[i]
                sel[pi].append((o, r))
            out = []
            for (pos, t), lst in zip(parts, sel):
                if not lst:
                    continue
                offs = torch.tensor([o for o, _ in lst], dtype=torch.int64)
                v = t if len(lst) == t.shape[0] and offs.tolist() == list(range(t.shape[0])) else t[offs.to(t.device)]
                out.append((torch.tensor([r for _, r in lst], dtype=torch.int64), v))
            self._device_write(self._set.upsert_parts, out)
            self._commit_rows(items, rows)
        return {"upserted_count": len(items)}

    def _plan_rows(self, items) -> list[int]:
        """Row of each (deduplicated) item: its existing row, or the next free rows; grows the
        shards if needed.  Registers nothing (see _commit_rows)."""
        rows, nxt = [], len(self._ids)
        for vid, _, _ in items:
            r = self._rows.get(vid)
            if r is None:
                r, nxt = nxt, nxt + 1
            rows.append(r)
        self._ensure_capacity(nxt)
        return rows

    def _commit_rows(self, items, rows) -> None:
        for (vid, _, md), r in zip(items, rows):
            if vid not in self._rows:
                self._rows[vid] = r
                self._ids.append(vid)
            self._meta[vid] = md
        self._gen += 1

    def _device_write(self, fn, *args) -> None:
        """A shard write under the lock.  If it raises part-way (an earlier shard already
        overwrote the rows of existing ids), the values cached by the last query no longer
        match the device: invalidate them before re-raising, so fetch reads the device."""
        try:
            fn(*args)
        except BaseException:
            self._gen += 1
            raise

    def _upsert_locked(self, items, vecs: torch.Tensor) -> None:
        # device write first: if it raises, no id is registered (no zero rows behind live ids)
        rows = self._plan_rows(items)
        self._device_write(self._set.upsert_rows, vecs, rows)
        self._commit_rows(items, rows)

    def query(self, vector=None, top_k: int = 10, include_values: bool = False, include_metadata: bool = False,
              id: str | None = None, namespace: str = "", **_: Any) -> dict:
        if vector is None and id is None:
            raise ValueError("query needs a vector or an id")
        if isinstance(top_k, bool) or int(top_k) != top_k or top_k < 1:
            raise ValueError("top_k must be a positive integer")
        top_k = int(top_k)
        if top_k > _lib.RC_TOPK_MAX:
            raise ValueError(f"top_k must be <= {_lib.RC_TOPK_MAX}")
        with self._mu:
            if vector is None:
                r = self._rows.get(id)
                if r is None:
                    return {"matches": [], "namespace": namespace}
                vector = self._set.fetch_rows([r])[0]
            q = _as_vector_np(vector, self.dimension)
            res = self._query_host_locked(q, top_k, include_values, include_metadata)[0]
        return {"matches": res, "namespace": namespace}

    def query_batch(self, vectors, top_k: int = 10, include_values: bool = False,
                    include_metadata: bool = False, mode: str = "auto") -> list[dict]:
        """Batched form of ``query`` (f16/bf16 shards run the MFMA path for >= 8 queries)."""
        if top_k < 1 or top_k > _lib.RC_TOPK_MAX:
            raise ValueError(f"top_k must be in [1, {_lib.RC_TOPK_MAX}]")
        if isinstance(vectors, torch.Tensor):
            q = vectors.to(torch.float32)
            if q.dim() != 2 or q.shape[1] != self.dimension:
                raise ValueError("queries must be [n, dimension]")
        else:
            q = torch.tensor([_as_vector(v, self.dimension) for v in vectors], dtype=torch.float32)
        with self._mu:
            res = self._query_locked(q, top_k, include_values, include_metadata, mode)
        return [{"matches": m, "namespace": ""} for m in res]

    def _query_locked(self, q: torch.Tensor, k: int, include_values: bool, include_metadata: bool,
                      mode: str = "auto") -> list[list[dict]]:
        n = len(self._ids)
        if n == 0 or q.shape[0] == 0:
            return [[] for _ in range(q.shape[0])]
        scores, rows = self._set.search(q, k, n, mode=mode)
        scores = scores.cpu().tolist()
        rows = rows.cpu().tolist()
        out = []
        recent: dict[str, np.ndarray] = {}
        for sq, rq in zip(scores, rows):
            sel = [(s, r) for s, r in zip(sq, rq) if r >= 0]
            vals = self._set.fetch_rows([r for _, r in sel]).numpy() if include_values and sel else None
            if vals is not None:
                recent.update((self._ids[r], v) for (_, r), v in zip(sel, vals))
            matches = []
            for j, (s, r) in enumerate(sel):
                vid = self._ids[r]
                m = Record(vals[j], id=vid, score=float(s)) if include_values else {"id": vid, "score": float(s)}
                if include_metadata:
                    dict.__setitem__(m, "metadata", dict(self._meta.get(vid, {})))
                matches.append(m)
            out.append(matches)
        if include_values:
            self._recent = (self._gen, recent)
        return out

    def _query_host_locked(self, q: np.ndarray, k: int, include_values: bool, include_metadata: bool) -> list[list[dict]]:
        """The request path (a query or a few): ``ShardSet.query_host``, one library call, the
        lists and (include_values) the matched rows' values come back together."""
        n = len(self._ids)
        if n == 0:
            return [[] for _ in range(q.shape[0])]
        sc, rw, val = self._set.query_host(q, k, n, include_values)
        out = []
        recent: dict[str, np.ndarray] = {}
        ids, meta = self._ids, self._meta
        for qi in range(q.shape[0]):
            rows = rw[qi].tolist()
            live = k - rows.count(-1)  # the lists are sorted: empty slots (-1) come last
            scores = sc[qi, :live].tolist()
            if include_values:
                # the reused host buffer is copied once (one memcpy); each match keeps its row as f32
                # and builds the Python list only if read (Record)
                vals = val[qi, :live].copy()
                matches = []
                for j in range(live):
                    vid = ids[rows[j]]
                    m = Record(vals[j], id=vid, score=scores[j])
                    recent[vid] = vals[j]
                    if include_metadata:
                        dict.__setitem__(m, "metadata", dict(meta.get(vid, {})))
                    matches.append(m)
            else:
                matches = [{"id": ids[r], "score": s} for s, r in zip(scores, rows[:live])]
                if include_metadata:
                    for m in matches:
                        m["metadata"] = dict(meta.get(m["id"], {}))
            out.append(matches)
        if include_values:
            self._recent = (self._gen, recent)
        return out

    def fetch(self, ids: Sequence[str], namespace: str = "") -> dict:
        with self._mu:
            found = [(i, self._rows[i]) for i in ids if i in self._rows]
            vectors = {}
            gen, recent = self._recent
            if found and gen == self._gen and all(i in recent for i, _ in found):
                vals = [recent[i] for i, _ in found]  # fetched by the query just before: no second device read
            elif found:
                vals = self._set.fetch_rows([r for _, r in found]).numpy()
            if found:
                for (vid, _), v in zip(found, vals):
                    rec = Record(v, id=vid)  # "values" becomes a list when read (retriever/main.py reads metadata)
                    dict.__setitem__(rec, "metadata", dict(self._meta.get(vid, {})))
                    vectors[vid] = rec
        return {"vectors": vectors, "namespace": namespace}

    # ---------------------------------------------------------- persistence --
    # Pinecone keeps an index durable server-side (the reference only opens it by
    # name, ingesting/utils.py:23-38); the in-HBM index is saved to a directory:
    # manifest.json (name, dimension, dtype, ids in row order, metadata) +
    # rows.npy (raw stored bytes in GLOBAL row order, exactly what search scores;
    # independent of the shard count) + norms.npy.
    SNAPSHOT_FORMAT = 1

    def save(self, path: str) -> None:
        import numpy as np

        with self._mu:
            os.makedirs(path, exist_ok=True)
            n = len(self._ids)
            rows, norms = self._set.export_rows(n)
            np.save(os.path.join(path, "rows.npy"), rows)
            np.save(os.path.join(path, "norms.npy"), norms)
            manifest = {"format": self.SNAPSHOT_FORMAT, "name": self.name, "dimension": self.dimension,
                        "metric": self.metric, "dtype": self._set.dtype, "ld": self._set.ld, "count": n,
                        "capacity": self._set.capacity, "filter": self._set.filter,
                        "ids": list(self._ids), "metadata": {i: self._meta.get(i, {}) for i in self._ids}}
            tmp = os.path.join(path, "manifest.json.tmp")
            with open(tmp, "w") as f:
                json.dump(manifest, f)
            os.replace(tmp, os.path.join(path, "manifest.json"))  # the manifest lands last

    @classmethod
    def load(cls, path: str, capacity: int | None = None, device=None, shards: int | None = None,
             devices=None, filter: str | None = None) -> "Index":
        import numpy as np

        with open(os.path.join(path, "manifest.json")) as f:
            man = json.load(f)
        if man.get("format") != cls.SNAPSHOT_FORMAT:
            raise ValueError(f"unsupported snapshot format {man.get('format')!r}")
        n = int(man["count"])
        idx = cls(man["name"], dimension=man["dimension"], metric=man["metric"], dtype=man["dtype"],
                  capacity=max(int(capacity or man.get("capacity", 0)), n, 1), device=device, shards=shards,
                  devices=devices, filter=filter or man.get("filter", "native"))
        if idx._set.ld != man["ld"]:
            raise ValueError("snapshot row layout does not match this build")
        rows = np.load(os.path.join(path, "rows.npy"), allow_pickle=False)
        norms = np.load(os.path.join(path, "norms.npy"), allow_pickle=False)
        if rows.shape[0] != n or norms.shape[0] != n or len(man["ids"]) != n:
            raise ValueError("snapshot files disagree on the vector count")
        if n:
            idx._set.import_rows(rows, norms)
        idx._ids = list(man["ids"])
        idx._rows = {vid: r for r, vid in enumerate(idx._ids)}
        idx._meta = {vid: dict(man["metadata"].get(vid, {})) for vid in idx._ids}
        return idx

    def describe_index_stats(self) -> dict:
        return {"dimension": self.dimension, "index_fullness": len(self._ids) / self._set.capacity,
                "total_vector_count": len(self._ids), "namespaces": {"": {"vector_count": len(self._ids)}},
                "shards": self._set.n}
