"""The C-ABI library loads on a CPU-only host and exports every entry point of include/*.h.

No compute calls: only argument validation paths that return before touching HIP.
"""
import ctypes
import os
import re

import pytest

from conftest import REPO, import_pkg

HEADER = os.path.join(REPO, "include", "retrieval_core.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rc_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    return import_pkg("_lib").load()


def test_header_declares_the_abi():
    names = declared_functions()
    assert "rc_index_search" in names and "rc_embed" in names and "rc_topk_merge" in names
    assert len(names) >= 20


def test_library_exports_every_declared_symbol(lib):
    raw = ctypes.CDLL(import_pkg("_lib").LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(raw, n)]
    assert missing == []
    assert getattr(lib, "rc_missing_symbols", ()) == ()


def test_python_binding_covers_the_header():
    sigs = import_pkg("_lib").SIGNATURES
    assert set(declared_functions()) <= set(sigs)


def test_abi_version(lib):
    assert lib.rc_abi_version() == 1


def test_invalid_arguments_rejected_before_any_device_call(lib):
    L = import_pkg("_lib")
    h = ctypes.c_void_p()
    st = lib.rc_index_create(0, 0, L.RC_F32, 10, 0, ctypes.byref(h))
    assert st == L.RC_ERR_INVALID
    assert b"dimension" in lib.rc_last_error()
    st = lib.rc_index_create(0, 768, 7, 10, 0, ctypes.byref(h))
    assert st == L.RC_ERR_INVALID
    st = lib.rc_index_create(0, 4096, L.RC_F32, 10, 0, ctypes.byref(h))
    assert st == L.RC_ERR_UNSUPPORTED
    st = lib.rc_topk_merge(None, None, 0, 1, 5, 5, None, None, None)
    assert st == L.RC_ERR_INVALID
    cfg = L.VitConfig(224, 16, 512, 12, 8, 3072, 1e-6, 4)
    m = ctypes.c_void_p()
    assert lib.rc_model_create(0, ctypes.byref(cfg), ctypes.byref(m)) == L.RC_ERR_UNSUPPORTED


def test_check_maps_status_to_exceptions(lib):
    L = import_pkg("_lib")
    h = ctypes.c_void_p()
    with pytest.raises(ValueError):
        L.check(lib.rc_index_create(0, -1, L.RC_F32, 10, 0, ctypes.byref(h)))
    L.check(L.RC_OK)
