"""Loader for the CPU parity checker (oracle/compose_ref.c, oracle/crdt_ref.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, ``__graft_entry__.smoke()`` and
bench.py's cpu_baseline leg.  The product package never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Tuple

import numpy as np

from semantic_merge_amd._abi import SmxComposeOut, SmxOps, SmxRgaOps, SmxRgaOut
from semantic_merge_amd.marshal import SoA

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libsmx_oracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _lib.smx_oracle_compose.argtypes = [C.POINTER(SmxOps), C.POINTER(SmxComposeOut)]
        _lib.smx_oracle_compose.restype = C.c_int
        _lib.smx_oracle_rga.argtypes = [C.POINTER(SmxRgaOps), C.POINTER(SmxRgaOut)]
        _lib.smx_oracle_rga.restype = C.c_int
    return _lib


def _p(a: np.ndarray) -> int:
    return a.ctypes.data


def compose(soa: SoA) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
    """Reference-order composition of ``soa`` on the CPU.

    Returns (order, addr, file, ctx, conflict_pairs[n, 2]) trimmed to the counts."""
    n = soa.n
    arrs = [np.ascontiguousarray(x) for x in
            (soa.kind, soa.ts, soa.oid_hi, soa.oid_lo, soa.sym, soa.v0, soa.v1)]
    ops = SmxOps(soa.n_a, soa.n_b, soa.n_sym, *[_p(a) for a in arrs])
    order = np.empty(max(n, 1), np.int32)
    addr = np.empty(max(n, 1), np.int32)
    file = np.empty(max(n, 1), np.int32)
    ctx = np.empty(max(n, 1), np.int32)
    cap = max(min(soa.n_a, soa.n_b), 1)
    conf = np.empty(2 * cap, np.int32)
    counts = np.zeros(2, np.int64)
    out = SmxComposeOut(_p(order), _p(addr), _p(file), _p(ctx), _p(conf), cap, _p(counts))
    rc = lib().smx_oracle_compose(C.byref(ops), C.byref(out))
    if rc != 0:
        raise RuntimeError(f"oracle compose failed: {rc}")
    k, nc = int(counts[0]), int(counts[1])
    return order[:k], addr[:k], file[:k], ctx[:k], conf[: 2 * nc].reshape(nc, 2)


def rga(n_lists: int, list_id, op, value, anchor, t, author, opid_hi, opid_lo):
    """Sequential RGA replay; returns (values, src, offsets)."""
    arrs = [np.ascontiguousarray(a, dtype=d) for a, d in (
        (list_id, np.uint32), (op, np.uint8), (value, np.uint32), (anchor, np.uint32),
        (t, np.int64), (author, np.uint32), (opid_hi, np.uint64), (opid_lo, np.uint64))]
    n = len(arrs[0])
    ops = SmxRgaOps(n, n_lists, *[_p(a) for a in arrs])
    vals = np.empty(max(n, 1), np.uint32)
    src = np.empty(max(n, 1), np.int32)
    offs = np.empty(n_lists + 1, np.int64)
    counts = np.zeros(1, np.int64)
    out = SmxRgaOut(_p(vals), _p(src), _p(offs), _p(counts))
    rc = lib().smx_oracle_rga(C.byref(ops), C.byref(out))
    if rc != 0:
        raise RuntimeError(f"oracle rga failed: {rc}")
    k = int(counts[0])
    return vals[:k], src[:k], offs
