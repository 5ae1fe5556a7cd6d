"""ctypes mirror of include/smx.h (structs and prototypes).

Shared by the product loader (``_lib.py``) and, in tests, by the CPU oracle
loader (``oracle/oracle.py``): both libraries use the same structs.
"""
from __future__ import annotations

import ctypes as C

c_i64p = C.POINTER(C.c_int64)


class SmxOps(C.Structure):
    _fields_ = [
        ("n_a", C.c_int64),
        ("n_b", C.c_int64),
        ("n_sym", C.c_int64),
        ("kind", C.c_void_p),
        ("ts", C.c_void_p),
        ("oid_hi", C.c_void_p),
        ("oid_lo", C.c_void_p),
        ("sym", C.c_void_p),
        ("v0", C.c_void_p),
        ("v1", C.c_void_p),
        ("b_gap", C.c_int64),
    ]


class SmxComposeOut(C.Structure):
    _fields_ = [
        ("order", C.c_void_p),
        ("addr", C.c_void_p),
        ("file", C.c_void_p),
        ("ctx", C.c_void_p),
        ("conflicts", C.c_void_p),
        ("conflict_cap", C.c_int64),
        ("counts", C.c_void_p),
    ]


class SmxShard(C.Structure):
    _fields_ = [
        ("rank", C.c_int32),
        ("world", C.c_int32),
        ("src_a", C.c_int64),
        ("src_b", C.c_int64),
        ("halo_n", C.c_int64 * 2),
        ("halo_more", C.c_int32 * 2),
        ("halo_sym", C.c_void_p * 2),
        ("halo_cls", C.c_void_p * 2),
        ("halo_src", C.c_void_p * 2),
        ("in_ahead", C.c_int32),
        ("in_d", C.c_int64),
        ("summary", C.c_void_p),
        ("halo_cap", C.c_int64),
        ("export_sym", C.c_void_p),
        ("export_cls", C.c_void_p),
        ("export_src", C.c_void_p),
        ("part_tab", C.c_void_p),
        ("fin_tab", C.c_void_p),
        ("glob", C.c_void_p),
        ("mv_prefix", C.c_void_p),
        ("halo_dev", C.c_void_p),
        ("in_state_dev", C.c_void_p),
        ("src_map", C.c_void_p),
        ("summary_host", C.c_void_p),
        ("order_gather", C.c_void_p),
        ("tab32", C.c_int32),
    ]


SHARD_ORDER, SHARD_WALK, SHARD_TABLES, SHARD_EMIT = 0, 1, 2, 3
SHARD_ORDER_FIX = 4
SHARD_SCATTER = 5
PLAN_NAMES = ("presorted", "segmented", "radix", "radix+oid_lo", "presorted-wide", "small")  # smx_last_plan()
SHARD_SUMMARY = 32


class SmxRgaOps(C.Structure):
    _fields_ = [
        ("n_ops", C.c_int64),
        ("n_lists", C.c_int64),
        ("list", C.c_void_p),
        ("op", C.c_void_p),
        ("value", C.c_void_p),
        ("anchor", C.c_void_p),
        ("t", C.c_void_p),
        ("author", C.c_void_p),
        ("opid_hi", C.c_void_p),
        ("opid_lo", C.c_void_p),
    ]


class SmxRgaOut(C.Structure):
    _fields_ = [
        ("out_value", C.c_void_p),
        ("out_src", C.c_void_p),
        ("out_offsets", C.c_void_p),
        ("counts", C.c_void_p),
        ("out_tomb", C.c_void_p),
    ]


# Every symbol include/smx.h declares (tests check the built library exports them).
RGA_GROUPED = 1   # smx_rga_replay_ex flag (include/smx.h SMX_RGA_GROUPED)

EXPORTS = (
    "smx_compose_workspace_bytes",
    "smx_compose",
    "smx_compose_async",
    "smx_compose_finish",
    "smx_release_graphs",
    "smx_last_plan",
    "smx_set_small_limit",
    "smx_shard_step",
    "smx_shard_range_info",
    "smx_set_profiling",
    "smx_set_profiling_stages",
    "smx_stage_times",
    "smx_stage_name",
    "smx_reset_stage_times",
    "smx_rga_workspace_bytes",
    "smx_rga_replay",
    "smx_rga_replay_ex",
    "smx_last_error",
    "smx_version",
)


def declare(lib: C.CDLL) -> C.CDLL:
    """Attach argtypes/restype for the product library."""
    lib.smx_compose_workspace_bytes.argtypes = [C.c_int64, C.c_int64, C.c_int64,
                                                C.POINTER(C.c_size_t)]
    lib.smx_compose_workspace_bytes.restype = C.c_int
    lib.smx_compose.argtypes = [C.POINTER(SmxOps), C.POINTER(SmxComposeOut), C.c_void_p,
                                C.c_size_t, C.c_void_p]
    lib.smx_compose.restype = C.c_int
    for f in ("smx_compose_async", "smx_compose_finish"):
        getattr(lib, f).argtypes = lib.smx_compose.argtypes
        getattr(lib, f).restype = C.c_int
    lib.smx_release_graphs.argtypes = [C.c_void_p]
    lib.smx_release_graphs.restype = C.c_int
    lib.smx_last_plan.argtypes = []
    lib.smx_last_plan.restype = C.c_int
    lib.smx_set_small_limit.argtypes = [C.c_int64]
    lib.smx_set_small_limit.restype = C.c_int64
    lib.smx_shard_step.argtypes = [C.POINTER(SmxOps), C.POINTER(SmxShard), C.POINTER(SmxComposeOut),
                                   C.c_void_p, C.c_size_t, C.c_void_p, C.c_int]
    lib.smx_shard_step.restype = C.c_int
    if hasattr(lib, "smx_shard_range_info"):  # (older builds, e.g. A/B baselines, lack it)
        lib.smx_shard_range_info.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_int32,
                                             C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]
        lib.smx_shard_range_info.restype = C.c_int
    lib.smx_set_profiling.argtypes = [C.c_int]
    lib.smx_set_profiling.restype = C.c_int
    lib.smx_set_profiling_stages.argtypes = [C.c_uint32]
    lib.smx_set_profiling_stages.restype = C.c_int
    lib.smx_stage_times.argtypes = [C.POINTER(C.c_double), c_i64p, C.c_int]
    lib.smx_stage_times.restype = C.c_int
    lib.smx_stage_name.argtypes = [C.c_int]
    lib.smx_stage_name.restype = C.c_char_p
    lib.smx_reset_stage_times.argtypes = []
    lib.smx_reset_stage_times.restype = C.c_int
    lib.smx_rga_workspace_bytes.argtypes = [C.c_int64, C.c_int64, C.POINTER(C.c_size_t)]
    lib.smx_rga_workspace_bytes.restype = C.c_int
    lib.smx_rga_replay.argtypes = [C.POINTER(SmxRgaOps), C.POINTER(SmxRgaOut), C.c_void_p,
                                   C.c_size_t, C.c_void_p]
    lib.smx_rga_replay.restype = C.c_int
    lib.smx_rga_replay_ex.argtypes = [C.POINTER(SmxRgaOps), C.POINTER(SmxRgaOut), C.c_void_p,
                                      C.c_size_t, C.c_uint32, C.c_void_p]
    lib.smx_rga_replay_ex.restype = C.c_int
    lib.smx_last_error.argtypes = []
    lib.smx_last_error.restype = C.c_char_p
    lib.smx_version.argtypes = []
    lib.smx_version.restype = C.c_char_p
    return lib
