"""ctypes binding of ``lib/libretrieval_core.so`` (the C ABI in ``include/retrieval_core.h``).

The library is loaded after ``torch`` so that it binds to the HIP runtime
torch already mapped (both carry SONAME ``libamdhip64.so.7``) — one runtime,
one device context, and torch tensors' ``data_ptr()`` are valid device
pointers for every call.  There is no fallback: if the library is missing the
import fails loudly with instructions to build it.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch  # noqa: F401  (must be loaded before the HIP library, see above)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# RC_LIB_PATH: diagnostic builds only (tools/build_diag.sh); the product loads the in-tree library
LIB_PATH = os.environ.get("RC_LIB_PATH") or os.path.join(PKG_DIR, "lib", "libretrieval_core.so")

RC_OK = 0
RC_ERR_INVALID = 1
RC_ERR_HIP = 2
RC_ERR_OOM = 3
RC_ERR_UNSUPPORTED = 4
RC_ERR_STATE = 5

RC_F32, RC_F16, RC_BF16 = 0, 1, 2
RC_TOPK_MAX = 256
RC_SEARCH_AUTO, RC_SEARCH_SCAN, RC_SEARCH_MFMA = 0, 1, 2
SEARCH_MODES = {"auto": RC_SEARCH_AUTO, "scan": RC_SEARCH_SCAN, "mfma": RC_SEARCH_MFMA}
DTYPES = {"float32": RC_F32, "f32": RC_F32, "float16": RC_F16, "f16": RC_F16, "bfloat16": RC_BF16, "bf16": RC_BF16}
RC_FILTER_NATIVE, RC_FILTER_I8 = 0, 1
FILTERS = {"native": RC_FILTER_NATIVE, "i8": RC_FILTER_I8}


class RetrievalCoreError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[rc status {code}] {msg}")
        self.code = code


class RetrievalCoreValueError(RetrievalCoreError, ValueError):
    pass


class VitConfig(C.Structure):
    _fields_ = [
        ("image_size", C.c_int),
        ("patch", C.c_int),
        ("hidden", C.c_int),
        ("layers", C.c_int),
        ("heads", C.c_int),
        ("mlp", C.c_int),
        ("ln_eps", C.c_float),
        ("max_batch", C.c_int),
    ]


class JpegInfo(C.Structure):
    _fields_ = [
        ("width", C.c_int32),
        ("height", C.c_int32),
        ("ncomp", C.c_int32),
        ("supported", C.c_int32),
        ("hmax", C.c_int32),
        ("vmax", C.c_int32),
        ("restart_interval", C.c_int32),
        ("mcux", C.c_int32),
        ("mcuy", C.c_int32),
        ("h", C.c_int32 * 3),
        ("v", C.c_int32 * 3),
        ("bw", C.c_int32 * 3),
        ("bh", C.c_int32 * 3),
        ("blocks", C.c_int64),
    ]


_vp = C.c_void_p
_i64 = C.c_int64
_i32 = C.c_int
_pi64 = C.POINTER(C.c_int64)
_pi32 = C.POINTER(C.c_int)
_pd = C.POINTER(C.c_double)
_pf = C.POINTER(C.c_float)

# name -> (restype, argtypes)
SIGNATURES = {
    "rc_last_error": (C.c_char_p, []),
    "rc_abi_version": (C.c_int, []),
    "rc_alloc_count": (C.c_int64, []),
    "rc_index_create": (C.c_int, [_i32, _i32, _i32, _i64, _i64, C.POINTER(_vp)]),
    "rc_index_destroy": (C.c_int, [_vp]),
    "rc_index_info": (C.c_int, [_vp, _pi32, _pi32, _pi64, _pi64]),
    "rc_index_data": (C.c_int, [_vp, C.POINTER(_vp), C.POINTER(_vp)]),
    "rc_index_reserve": (C.c_int, [_vp, _i32, _i32]),
    "rc_index_upsert": (C.c_int, [_vp, _vp, _i64, _vp, _vp]),
    "rc_index_fetch": (C.c_int, [_vp, _vp, _i64, _vp, _vp]),
    "rc_index_fetch_stored": (C.c_int, [_vp, _vp, _i64, _vp, _vp]),
    "rc_index_search": (C.c_int, [_vp, _vp, _i32, _i64, _i32, _vp, _vp, _vp]),
    "rc_index_export": (C.c_int, [_vp, _i64, _i64, _vp, _vp, _vp]),
    "rc_index_import": (C.c_int, [_vp, _i64, _i64, _vp, _vp, _vp]),
    "rc_index_search_ex": (C.c_int, [_vp, _vp, _i32, _i64, _i32, _vp, _vp, _i32, _vp]),
    "rc_index_gemm_timing_read": (C.c_int, [_vp, _pd, _pi64, _pd, _pi64]),
    "rc_index_fill_random": (C.c_int, [_vp, C.c_uint64, _i64, _i64, _vp]),
    "rc_topk_merge": (C.c_int, [_vp, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp]),
    "rc_index_set_row_map": (C.c_int, [_vp, _i64, _i64]),
    "rc_index_grow": (C.c_int, [_vp, _i64, _vp]),
    "rc_index_set_filter": (C.c_int, [_vp, _i32, _vp]),
    "rc_index_get_filter": (C.c_int, [_vp, _pi32]),
    "rc_sharded_set_filter": (C.c_int, [_vp, _i32]),
    "rc_sharded_create": (C.c_int, [_i32, _pi32, _i32, _i32, _i64, C.POINTER(_vp)]),
    "rc_sharded_destroy": (C.c_int, [_vp]),
    "rc_sharded_force_remote": (C.c_int, [_vp]),
    "rc_sharded_info": (C.c_int, [_vp, _pi32, _pi64, _pi64]),
    "rc_sharded_shard": (C.c_int, [_vp, _i32, C.POINTER(_vp)]),
    "rc_sharded_grow": (C.c_int, [_vp, _i64]),
    "rc_sharded_upsert": (C.c_int, [_vp, _vp, _i64, _vp, _vp]),
    "rc_sharded_fetch": (C.c_int, [_vp, _vp, _i64, _vp, _i32]),
    "rc_sharded_search": (C.c_int, [_vp, _vp, _i32, _i64, _i32, _vp, _vp, _i32, _vp]),
    "rc_sharded_query_host": (C.c_int, [_vp, _vp, _i32, _i64, _i32, _i32, _vp, _vp, _vp]),
    "rc_index_timing": (C.c_int, [_vp, _i32]),
    "rc_index_timing_read": (C.c_int, [_vp, _pd, _pi64, _pd]),
    "rc_model_create": (C.c_int, [_i32, C.POINTER(VitConfig), C.POINTER(_vp)]),
    "rc_model_destroy": (C.c_int, [_vp]),
    "rc_model_set_weight": (C.c_int, [_vp, C.c_char_p, _vp, _i64]),
    "rc_model_set_preprocess": (C.c_int, [_vp, _i32, C.c_double, _pf, _pf]),
    "rc_model_finalize": (C.c_int, [_vp]),
    "rc_embed": (C.c_int, [_vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp]),
    "rc_preprocess": (C.c_int, [_vp, _vp, _i32, _i32, _i32, _vp, _vp]),
    "rc_model_set_parts": (C.c_int, [_vp, _i32]),
    "rc_model_set_last_layer": (C.c_int, [_vp, _i32]),
    "rc_model_set_ln_fold": (C.c_int, [_vp, _i32]),
    "rc_model_set_graphs": (C.c_int, [_vp, _i32]),
    "rc_model_timing": (C.c_int, [_vp, _i32]),
    "rc_model_timing_read": (C.c_int, [_vp, _i32, _pd, _pi64, _pd]),
    "rc_model_timing_reset": (C.c_int, [_vp]),
    "rc_gemm_bf16": (C.c_int, [_i32, _i32, _vp, _vp, _vp, _i32, _i32, _i32, _vp, _vp, _i32, _vp]),
    "rc_jpeg_probe": (C.c_int, [C.c_char_p, _i64, C.POINTER(JpegInfo)]),
    "rc_jpeg_decode_coefficients": (C.c_int, [C.c_char_p, _i64, _vp, _vp]),
    "rc_jpeg_decoder_create": (C.c_int, [_i32, _i32, _i64, C.POINTER(_vp)]),
    "rc_jpeg_decoder_destroy": (C.c_int, [_vp]),
    "rc_jpeg_decode": (C.c_int, [_vp, _i32, C.POINTER(C.c_char_p), _pi64, _vp, _pi64, _vp]),
    "rc_jpeg_decode_resized": (C.c_int, [_vp, _i32, C.POINTER(C.c_char_p), _pi64, _i32, _i32, _vp, _vp]),
}

# diagnostic builds only (tools/build_diag.sh, loaded with RC_LIB_PATH): bound when present,
# never required of the product library
DIAG_SIGNATURES = {
    "rc_diag_set_gemm_variant": (C.c_int, [_vp, _i32]),
    "rc_diag_set_stamps": (C.c_int, [_vp]),
    "rc_diag_set_attention": (C.c_int, [_vp, _i32]),
    "rc_diag_set_skinny_wpb": (C.c_int, [_vp, _i32]),
    "rc_diag_set_part_priority": (C.c_int, [_vp, _i32]),
    "rc_diag_set_group_m": (C.c_int, [_vp, _i32]),
    "rc_diag_set_band_skip": (C.c_int, [_i32]),
    "rc_diag_set_filter_split": (C.c_int, [_i32]),
    "rc_diag_set_filter_aux": (C.c_int, [_i32]),
}

_lock = threading.Lock()
_lib = None


def load() -> C.CDLL:
    """Open the library once (raises if it was not built)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build the HIP library first "
                "(python -c 'import __graft_entry__ as g; g.build()' or python <pkg>/build.py)"
            )
        lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        missing = []
        for name, (res, args) in SIGNATURES.items():
            try:
                fn = getattr(lib, name)
            except AttributeError:
                missing.append(name)
                continue
            fn.restype = res
            fn.argtypes = args
        for name in missing:  # fail loudly at the first call, never silently

            def _missing(*_a, _n=name):
                raise ImportError(f"{LIB_PATH} does not export {_n}: rebuild the library")

            setattr(lib, name, _missing)
        for name, (res, args) in DIAG_SIGNATURES.items():
            fn = getattr(lib, name, None)
            if fn is not None:
                fn.restype = res
                fn.argtypes = args
        lib.rc_missing_symbols = tuple(missing)
        if lib.rc_abi_version() != 1:
            raise ImportError("libretrieval_core ABI version mismatch")
        _lib = lib
        return lib


def check(status: int) -> None:
    if status == RC_OK:
        return
    msg = load().rc_last_error().decode("utf-8", "replace")
    if status in (RC_ERR_INVALID, RC_ERR_UNSUPPORTED):
        raise RetrievalCoreValueError(status, msg)
    raise RetrievalCoreError(status, msg)


def stream_ptr(stream: "torch.cuda.Stream | None" = None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def ptr(t: "torch.Tensor | None") -> int | None:
    if t is None:
        return None
    return int(t.data_ptr())
