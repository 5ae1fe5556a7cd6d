"""Host materialiser: device result arrays -> fresh ``Op`` / ``Conflict`` objects.

The device reports, per emitted op (in output order): the source index into
``A || B`` and three string ids (-1 = none): the symbol's move-chain
``newAddress`` and ``newFile`` visible to that op, and its rename context.
This module applies them exactly as ``semmerge/compose.py:30-49`` does to a
``_clone_op`` copy (``compose.py:117-127``: four independent ``deepcopy``s),
preserving dict key order, so ``to_dict()`` JSON is byte-identical.
"""
from __future__ import annotations

import dataclasses
from copy import deepcopy
from typing import Any, List, Sequence, Tuple

import numpy as np

from .conflict import divergent_rename
from .ops import KIND_MOVE, KIND_RENAME


def materialize_ops(ops: Sequence[Any], kind: np.ndarray, strings: Sequence[str],
                    order: np.ndarray, addr: np.ndarray, file: np.ndarray,
                    ctx: np.ndarray) -> List[Any]:
    out: List[Any] = []
    order_l = order.tolist()
    addr_l = addr.tolist()
    file_l = file.tolist()
    ctx_l = ctx.tolist()
    kind_l = kind.tolist()
    for t, src in enumerate(order_l):
        op = ops[src]
        tgt = op.target
        tcls = type(tgt)
        clone = type(op)(
            id=op.id,
            schemaVersion=op.schemaVersion,
            type=op.type,
            target=tcls(symbolId=tgt.symbolId, addressId=tgt.addressId),
            params=deepcopy(op.params),
            guards=deepcopy(op.guards),
            effects=deepcopy(op.effects),
            provenance=deepcopy(op.provenance),
        )
        k = kind_l[src]
        a, f, c = addr_l[t], file_l[t], ctx_l[t]
        if k == KIND_MOVE:
            if a >= 0:
                clone.params["newAddress"] = strings[a]
            if f >= 0:
                clone.params["newFile"] = strings[f]
        if a >= 0:
            clone.target = tcls(symbolId=tgt.symbolId, addressId=strings[a])
        if k == KIND_RENAME and f >= 0:
            clone.params["newFile"] = strings[f]
            clone.params["file"] = strings[f]
        if c >= 0 and k != KIND_RENAME:
            clone.params = {**clone.params, "renameContext": strings[c]}
        out.append(clone)
    return out


def materialize_ops_native(ops: Sequence[Any], kind: np.ndarray, strings: Sequence[str],
                           order: np.ndarray, addr: np.ndarray, file: np.ndarray,
                           ctx: np.ndarray) -> List[Any]:
    """``materialize_ops`` done by the native host module (csrc/smx_host.cpp)."""
    from ._host import host

    def i32(a):
        return np.ascontiguousarray(a, dtype=np.int32)
    return host().materialize_ops(list(ops), np.ascontiguousarray(kind, dtype=np.uint8),
                                  list(strings), i32(order), i32(addr), i32(file), i32(ctx),
                                  KIND_MOVE, KIND_RENAME, deepcopy, smx_host_ctor_mode)


def smx_host_ctor_mode(cls: type, names: Tuple[str, ...]) -> int:
    """How the native materialiser may build ``cls(**dict(zip(names, values)))``.

    1 (2 when frozen): ``cls`` is a plain dataclass whose ``__init__`` is the one
    ``dataclasses`` generated for exactly ``names`` (every field in __init__, no
    ``__post_init__``, ``object.__new__``), so the constructor is ``object.__new__`` plus
    one ``setattr`` per field in order (``object.__setattr__`` when frozen) — what that
    generated code does.  0: anything else; the class is called.
    """
    if not dataclasses.is_dataclass(cls) or cls.__new__ is not object.__new__:
        return 0
    if hasattr(cls, "__post_init__"):
        return 0
    code = getattr(cls.__init__, "__code__", None)
    if code is None or code.co_filename != "<string>" or code.co_name != "__init__":
        return 0
    if code.co_kwonlyargcount or code.co_argcount != len(names) + 1:
        return 0
    if tuple(code.co_varnames[1:code.co_argcount]) != tuple(names):
        return 0
    if tuple(f.name for f in dataclasses.fields(cls)) != tuple(names):
        return 0
    return 2 if cls.__dataclass_params__.frozen else 1


_REF_DR = None


def conflict_factory():
    """The reference's own ``conflict_divergent_rename`` (semmerge/conflict.py:34-49) when
    the reference package is importable -- so callers get its ``Conflict`` class back --
    else this package's restatement (conflict.py here, same fields and payload)."""
    global _REF_DR
    if _REF_DR is None:
        try:
            from semmerge.conflict import conflict_divergent_rename as f
        except ImportError:
            f = divergent_rename
        _REF_DR = f
    return _REF_DR


def materialize_conflicts(ops: Sequence[Any], pairs: np.ndarray) -> List[Any]:
    """``pairs`` is an (n, 2) array of (A source index, B source index) in walk order."""
    make = conflict_factory()
    return [make(ops[a], ops[b]) for a, b in pairs.tolist()]
