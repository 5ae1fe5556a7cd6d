"""Loader for libsmx.so (the HIP library) and device-buffer plumbing.

PyTorch-ROCm is used only to own device memory and to name the current HIP
stream; every computation happens in libsmx's kernels through the C ABI of
include/smx.h.  There is no CPU fallback: without the library or a GPU these
functions raise.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Tuple

import numpy as np

from . import _abi
from .marshal import SoA

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SMX_LIB", os.path.join(HERE, "libsmx.so"))
_lib: Optional[C.CDLL] = None


class SmxError(RuntimeError):
    def __init__(self, code: int, msg: str) -> None:
        super().__init__(f"smx error {code}: {msg}")
        self.code = code


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libsmx.so not built at {LIB_PATH}; run __graft_entry__.build()")
        _lib = _abi.declare(C.CDLL(LIB_PATH))
    return _lib


def check(rc: int) -> None:
    if rc != 0:
        raise SmxError(rc, lib().smx_last_error().decode(errors="replace"))


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("semantic_merge_amd needs a ROCm GPU (torch.cuda.is_available() is False)")
    return torch


def _ptr(t) -> int:
    return t.data_ptr() if t is not None and t.numel() > 0 else 0


_hip: Optional[C.CDLL] = None


def _hiprt() -> C.CDLL:
    """The HIP runtime the process already runs (torch's, which libsmx shares: the same
    soname), for the session's two copies and its one stream sync -- a ctypes call each,
    against ~10 us of torch dispatch per copy_ / stream context on a 1k-op merge."""
    global _hip
    if _hip is None:
        _torch()
        lib()
        # the copy this process already mapped (torch's; libsmx resolved to it), by its
        # path: dlopen returns that same copy, never a second runtime
        path = None
        with open("/proc/self/maps") as fh:
            for line in fh:
                f = line.split()[-1] if line.strip() else ""
                if os.path.basename(f).startswith("libamdhip64.so"):
                    path = f
                    break
        if path is None:
            raise RuntimeError("the HIP runtime (libamdhip64) is not loaded in this process")
        h = C.CDLL(path)
        h.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
        h.hipMemcpyAsync.restype = C.c_int
        h.hipStreamSynchronize.argtypes = [C.c_void_p]
        h.hipStreamSynchronize.restype = C.c_int
        _hip = h
    return _hip


def _hip_check(rc: int, what: str) -> None:
    if rc != 0:
        raise SmxError(rc, f"{what} failed (hipError_t {rc})")


class DeviceCompose:
    """Device-resident inputs, outputs and workspace for repeated smx_compose calls."""

    def __init__(self, soa: SoA, device: str = "cuda") -> None:
        torch = _torch()
        self.torch = torch
        self.soa = soa
        self.n = soa.n
        dev = torch.device(device)
        self.device = dev

        def up(a, dt):
            return torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(dev, non_blocking=False)

        self.kind = up(soa.kind, np.uint8)
        self.ts = up(soa.ts, np.int64)      # bit-identical u64 payload
        self.hi = up(soa.oid_hi, np.int64)
        self.lo = up(soa.oid_lo, np.int64)
        self.sym = up(soa.sym, np.int32)
        self.v0 = up(soa.v0, np.int32)
        self.v1 = up(soa.v1, np.int32)
        n = max(self.n, 1)
        self.order = torch.empty(n, dtype=torch.int32, device=dev)
        self.addr = torch.empty(n, dtype=torch.int32, device=dev)
        self.file = torch.empty(n, dtype=torch.int32, device=dev)
        self.ctx = torch.empty(n, dtype=torch.int32, device=dev)
        self.cap = max(min(soa.n_a, soa.n_b), 1)
        self.conf = torch.empty(2 * self.cap, dtype=torch.int32, device=dev)
        self.counts = torch.zeros(2, dtype=torch.int64, device=dev)
        ws = C.c_size_t(0)
        check(lib().smx_compose_workspace_bytes(soa.n_a, soa.n_b, soa.n_sym, C.byref(ws)))
        self.ws_bytes = ws.value
        self.ws = torch.empty(max(ws.value, 1), dtype=torch.uint8, device=dev)
        self._ops = _abi.SmxOps(soa.n_a, soa.n_b, soa.n_sym, _ptr(self.kind), _ptr(self.ts),
                                _ptr(self.hi), _ptr(self.lo), _ptr(self.sym), _ptr(self.v0),
                                _ptr(self.v1))
        self._out = _abi.SmxComposeOut(_ptr(self.order), _ptr(self.addr), _ptr(self.file),
                                       _ptr(self.ctx), _ptr(self.conf), self.cap,
                                       _ptr(self.counts))

    def _args(self, stream):
        s = stream if stream is not None else self.torch.cuda.current_stream(self.device)
        return (C.byref(self._ops), C.byref(self._out), _ptr(self.ws), self.ws_bytes, s.cuda_stream)

    def run(self, stream=None) -> None:
        """One composition on `stream` (default: torch's current stream)."""
        check(lib().smx_compose(*self._args(stream)))

    def run_async(self, stream=None) -> None:
        """Enqueue the host-sync-free part (smx_compose_async; capturable in a graph)."""
        check(lib().smx_compose_async(*self._args(stream)))

    def finish(self, stream=None) -> None:
        """Complete what run_async left (smx_compose_finish: one stream sync)."""
        check(lib().smx_compose_finish(*self._args(stream)))

    @staticmethod
    def last_plan() -> str:
        return _abi.PLAN_NAMES[lib().smx_last_plan()]

    def results(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
        self.torch.cuda.synchronize(self.device)
        k, nc = (int(x) for x in self.counts.cpu().tolist())
        if k < 0:
            raise SmxError(-1, "invalid input: sym >= n_sym or kind >= 18")
        if nc > self.cap:
            raise SmxError(-2, f"{nc} conflicts exceed capacity {self.cap}")
        return (self.order[:k].cpu().numpy(), self.addr[:k].cpu().numpy(),
                self.file[:k].cpu().numpy(), self.ctx[:k].cpu().numpy(),
                self.conf[: 2 * nc].cpu().numpy().reshape(nc, 2))


def _al(x: int) -> int:
    return (x + 255) & ~255


class ComposeSession:
    """Reusable buffers for a stream of merges of any size (the drop-in's path): one
    pinned host staging area and one device area, grown on demand, never shrunk.  A
    merge is one host-to-device copy of the packed SoA columns, smx_compose, and one
    device-to-host copy of the outputs and counts -- no allocation after warm-up.
    `last` holds the host / device split of the last merge in seconds."""

    _IN = (("kind", 1), ("ts", 8), ("oid_hi", 8), ("oid_lo", 8), ("sym", 4), ("v0", 4), ("v1", 4))
    ASYNC_MAX = 1 << 22  # smx_compose_async + one sync below this many ops (SMX_EARLY_MIN)

    def __init__(self, device: str = "cuda") -> None:
        self.torch = _torch()
        self.device = self.torch.device(device)
        self.cap_n = self.cap_ws = -1
        self.last = {}
        self.busy = False  # results handed out as views are being read (dropin_session)
        # its own stream: repeated merges of one size replay the library's HIP graph
        self.stream = self.torch.cuda.Stream(self.device)

    _DT = {"kind": np.uint8, "ts": np.uint64, "oid_hi": np.uint64, "oid_lo": np.uint64, "sym": np.uint32,
           "v0": np.int32, "v1": np.int32}

    def staging(self, n: int) -> dict:
        """The input columns of an n-op merge as views of the pinned staging area, laid out
        as compose() copies it: a SoA marshalled into them is not packed again."""
        self._ensure(n, 0)
        hin = self.h_in.numpy()
        cols, off = {}, 0
        for name, w in self._IN:
            cols[name] = hin[off: off + n * w].view(self._DT[name])
            off += _al(n * w)
        return cols

    def _ensure(self, n: int, ws_bytes: int) -> None:
        torch = self.torch
        grown = n > self.cap_n or ws_bytes > self.cap_ws
        if n > self.cap_n:
            cap = max(n + n // 4, 1024)
            in_b = sum(_al(cap * w) for _, w in self._IN)
            out_b = 4 * _al(cap * 4) + _al(cap * 4) + 256     # 4 outputs, conflicts (2 * cap/2), counts
            self.h_in = torch.empty(in_b, dtype=torch.uint8, pin_memory=True)
            self.d_in = torch.empty(in_b, dtype=torch.uint8, device=self.device)
            self.h_out = torch.empty(out_b, dtype=torch.uint8, pin_memory=True)
            self.d_out = torch.empty(out_b, dtype=torch.uint8, device=self.device)
            self.cap_n = cap
        if ws_bytes > self.cap_ws:
            self.ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=self.device)
            self.cap_ws = ws_bytes
        if grown:  # new buffers come from the current stream's pool: ready before the session's stream uses them
            torch.cuda.synchronize(self.device)

    def compose(self, soa: SoA, copy: bool = True):
        """(order, addr, file, ctx, conflict_pairs) of one merge, computed on the GPU.
        copy=False: views of the session's pinned staging area, valid until its next merge
        (the drop-in materialises them at once)."""
        import time
        t0 = time.perf_counter()
        n = soa.n
        if n == 0:
            e = np.zeros(0, np.int32)
            return e, e, e, e, np.zeros((0, 2), np.int32)
        ws = C.c_size_t(0)
        check(lib().smx_compose_workspace_bytes(soa.n_a, soa.n_b, soa.n_sym, C.byref(ws)))
        self._ensure(n, ws.value)
        hin = self.h_in.numpy()
        off, ptrs = 0, {}
        d0 = self.d_in.data_ptr()
        h0 = hin.ctypes.data
        for name, w in self._IN:   # pack the columns into the pinned staging area (laid out for n)
            col = getattr(soa, name)
            if not (isinstance(col, np.ndarray) and col.ctypes.data == h0 + off and col.nbytes == n * w):
                hin[off: off + n * w] = np.ascontiguousarray(col).view(np.uint8).reshape(-1)
            ptrs[name] = d0 + off  # (a column marshalled into staging() is in place already)
            off += _al(n * w)
        t1 = time.perf_counter()
        hip = _hiprt()
        st = self.stream.cuda_stream
        _hip_check(hip.hipMemcpyAsync(d0, self.h_in.data_ptr(), off, 1, st), "hipMemcpyAsync (inputs)")
        ccap = max(min(soa.n_a, soa.n_b), 1)
        o0 = self.d_out.data_ptr()
        q = _al(n * 4)             # outputs laid out for n: one contiguous copy back
        ops = _abi.SmxOps(soa.n_a, soa.n_b, soa.n_sym, ptrs["kind"], ptrs["ts"], ptrs["oid_hi"],
                          ptrs["oid_lo"], ptrs["sym"], ptrs["v0"], ptrs["v1"])
        cnt_off = 4 * q + _al(8 * ccap)
        out = _abi.SmxComposeOut(o0, o0 + q, o0 + 2 * q, o0 + 3 * q, o0 + 4 * q, ccap, o0 + cnt_off)
        args = (C.byref(ops), C.byref(out), self.ws.data_ptr(), ws.value, st)
        hout = self.h_out.numpy()

        def copy_back():
            _hip_check(hip.hipMemcpyAsync(self.h_out.data_ptr(), o0, cnt_off + 16, 2, st), "hipMemcpyAsync (outputs)")
            _hip_check(hip.hipStreamSynchronize(st), "hipStreamSynchronize")
            return (int(x) for x in hout[cnt_off: cnt_off + 16].view(np.int64))
        if n < self.ASYNC_MAX:
            # merges below the early-verdict size: the asynchronous part, the copy back and
            # ONE stream sync; smx_compose_finish only when the counts ask for it (a plan
            # that failed, None-valued moves: counts[0] < -1)
            check(lib().smx_compose_async(*args))
            k, nc = copy_back()
            if k < -1:
                check(lib().smx_compose_finish(*args))
                k, nc = copy_back()
        else:  # (larger: the synchronous call, which waits for the plan's early verdict)
            check(lib().smx_compose(*args))
            k, nc = copy_back()
        t2 = time.perf_counter()
        if k < 0:
            raise SmxError(-1, "invalid input: sym >= n_sym or kind >= 18")
        if nc > ccap:
            raise SmxError(-2, f"{nc} conflicts exceed capacity {ccap}")
        res = tuple(hout[i * q: i * q + 4 * k].view(np.int32) for i in range(4))
        pairs = hout[4 * q: 4 * q + 8 * nc].view(np.int32).reshape(nc, 2)
        if copy:
            res, pairs = tuple(x.copy() for x in res), pairs.copy()
        self.last = {"pack_s": t1 - t0, "device_s": t2 - t1, "unpack_s": time.perf_counter() - t2}
        return res + (pairs,)


_sessions = {}


def session(device: str = "cuda") -> ComposeSession:
    """The calling thread's ComposeSession on `device`."""
    import threading
    key = (threading.get_ident(), str(device))
    s = _sessions.get(key)
    if s is None:
        s = _sessions[key] = ComposeSession(device)
    return s


class dropin_session:
    """The thread's session for one drop-in merge whose results are read as views of its
    staging area (marshal into it, compose, materialise): marked busy meanwhile, so that a
    merge started from inside that materialise -- a caller's Op class or deepcopy hook
    composing again -- gets buffers of its own instead of overwriting the views."""

    def __init__(self, device: str = "cuda") -> None:
        self.device = device

    def __enter__(self) -> ComposeSession:
        s = session(self.device)
        self.s = s if not s.busy else ComposeSession(self.device)
        self.s.busy = True
        return self.s

    def __exit__(self, *exc) -> None:
        self.s.busy = False


def compose_soa(soa: SoA, device: str = "cuda"):
    """(order, addr, file, ctx, conflict_pairs) of one merge, computed on the GPU
    (through the thread's reusable ComposeSession, or buffers of its own while a drop-in
    merge of this thread holds that session)."""
    s = session(device)
    return (s if not s.busy else ComposeSession(device)).compose(soa)


def set_small_limit(n: int) -> int:
    """Merges of at most n ops (0..2048) take the one-workgroup plan; returns the old limit."""
    return int(lib().smx_set_small_limit(int(n)))


def stage_times():
    """{stage: (total_ms, calls)} accumulated while smx_set_profiling(1)."""
    L = lib()
    ms = (C.c_double * 16)()
    calls = (C.c_int64 * 16)()
    n = L.smx_stage_times(ms, calls, 16)
    return {L.smx_stage_name(i).decode(): (ms[i], calls[i]) for i in range(n)}


def rga_replay_device(batch, device: str = "cuda", tombstones: bool = False, grouped: bool = False):
    """(values, src, offsets) of a batched RGA replay computed on the GPU; with
    tombstones=True the whole list state (live and tombstoned elements, crdt.py RGA.list)
    and a fourth array, the tombstone flags.  grouped=True: the batch's events come list
    by list (non-decreasing list ids, as crdt.marshal_streams builds them): the library
    skips its partition by list (it checks the claim and partitions when it is false)."""
    torch = _torch()
    dev = torch.device(device)
    n = batch.n
    if n == 0:
        e = (np.zeros(0, np.uint32), np.zeros(0, np.int32), np.zeros(batch.n_lists + 1, np.int64))
        return e + (np.zeros(0, np.bool_),) if tombstones else e

    def up(a, dt):
        return torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(dev)

    ins = [up(batch.list_id, np.int32), up(batch.op, np.uint8), up(batch.value, np.int32),
           up(batch.anchor, np.int32), up(batch.t, np.int64), up(batch.author, np.int32),
           up(batch.opid_hi, np.int64), up(batch.opid_lo, np.int64)]
    vals = torch.empty(n, dtype=torch.int32, device=dev)
    src = torch.empty(n, dtype=torch.int32, device=dev)
    offs = torch.empty(batch.n_lists + 1, dtype=torch.int64, device=dev)
    counts = torch.zeros(1, dtype=torch.int64, device=dev)
    tomb = torch.empty(n, dtype=torch.uint8, device=dev) if tombstones else None
    ws = C.c_size_t(0)
    check(lib().smx_rga_workspace_bytes(n, batch.n_lists, C.byref(ws)))
    wst = torch.empty(max(ws.value, 1), dtype=torch.uint8, device=dev)
    ops = _abi.SmxRgaOps(n, batch.n_lists, *[_ptr(t) for t in ins])
    out = _abi.SmxRgaOut(_ptr(vals), _ptr(src), _ptr(offs), _ptr(counts), _ptr(tomb))
    check(lib().smx_rga_replay_ex(C.byref(ops), C.byref(out), _ptr(wst), ws.value,
                                  _abi.RGA_GROUPED if grouped else 0,
                                  torch.cuda.current_stream(dev).cuda_stream))
    torch.cuda.synchronize(dev)
    k = int(counts.item())
    res = (vals[:k].cpu().numpy().view(np.uint32), src[:k].cpu().numpy(), offs.cpu().numpy())
    return res + (tomb[:k].cpu().numpy().astype(np.bool_),) if tombstones else res
