"""Host materialiser: device result arrays -> fresh ``Op`` / ``Conflict`` objects.

The device reports, per emitted op (in output order): the source index into
``A || B`` and three string ids (-1 = none): the symbol's move-chain
``newAddress`` and ``newFile`` visible to that op, and its rename context.
This module applies them exactly as ``semmerge/compose.py:30-49`` does to a
``_clone_op`` copy (``compose.py:117-127``: four independent ``deepcopy``s),
preserving dict key order, so ``to_dict()`` JSON is byte-identical.
"""
from __future__ import annotations

from copy import deepcopy
from typing import Any, List, Sequence

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


def materialize_conflicts(ops: Sequence[Any], pairs: np.ndarray) -> List[Any]:
    """``pairs`` is an (n, 2) array of (A source index, B source index) in walk order."""
    return [divergent_rename(ops[a], ops[b]) for a, b in pairs.tolist()]
