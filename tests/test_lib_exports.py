"""The C-ABI library builds for gfx950, loads, and exports every symbol include/smx.h declares."""
import ctypes
import os
import re

from semantic_merge_amd import _abi
from semantic_merge_amd._lib import LIB_PATH

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "smx.h")


def test_header_and_exports_agree():
    declared = set(re.findall(r"^(?:int|int64_t|const char\*)\s+(smx_\w+)\(", open(HDR).read(), re.M))
    assert declared == set(_abi.EXPORTS)


def test_library_exports_all_symbols():
    assert os.path.exists(LIB_PATH), "build libsmx.so first (__graft_entry__.build())"
    lib = ctypes.CDLL(LIB_PATH)
    for name in _abi.EXPORTS:
        assert hasattr(lib, name), name
    _abi.declare(lib)
    assert lib.smx_version().startswith(b"smx")
    size = ctypes.c_size_t(0)
    assert lib.smx_compose_workspace_bytes(1000, 1000, 10, ctypes.byref(size)) == 0
    assert size.value > 0
    assert lib.smx_compose_workspace_bytes(-1, 0, 0, ctypes.byref(size)) != 0
    assert lib.smx_last_error()


def test_code_object_targets_gfx950():
    data = open(LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_native_host_module_loads():
    from semantic_merge_amd._host import host
    h = host()
    for name in ("marshal_ops", "materialize_ops", "deep_copy"):
        assert callable(getattr(h, name)), name
