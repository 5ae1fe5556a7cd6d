"""Op-log decoding on the native host module: the data format on
the input side of compose.

* ``ops_from_dicts(items)`` is ``[Op.from_dict(d) for d in items]``
  (``semmerge/ops.py:89-100``): same coercions, same evaluation order, same exceptions.
  It runs in ``csrc/smx_host.cpp``. Plain dataclasses (the reference's ``Op`` and
  ``Target``) are built as their generated ``__init__`` would build them; any other
  class is called.
* ``oplog_from_json(text)`` is ``OpLog.from_json`` (``ops.py:116-118``): a JSON parse,
  then ``ops_from_dicts``.
* ``ops_from_worker_result(result)`` is what ``TSWorker.build_and_diff`` does with the
  worker's JSON-RPC result (``semmerge/lang/ts/bridge.py:36-40``).

Pass the reference's own classes as ``op_cls`` / ``target_cls`` to get its ``Op``
objects back.
"""
from __future__ import annotations

import json
from typing import Any, Dict, List, Sequence, Tuple

from ._host import host
from .materialize import smx_host_ctor_mode
from .ops import Op, Target


def ops_from_dicts(items: Sequence[Any], op_cls: type = Op, target_cls: type = Target) -> List[Any]:
    return host().ops_from_dicts(list(items), op_cls, target_cls, smx_host_ctor_mode)


def oplog_from_json(data: str, op_cls: type = Op, target_cls: type = Target) -> List[Any]:
    return ops_from_dicts(json.loads(data), op_cls, target_cls)


def ops_from_worker_result(result: Dict[str, Any], op_cls: type = Op,
                           target_cls: type = Target) -> Tuple[List[Any], List[Any], Any]:
    """(opLogLeft ops, opLogRight ops, symbolMaps) of a ``buildAndDiff`` result."""
    return (ops_from_dicts(result.get("opLogLeft", []), op_cls, target_cls),
            ops_from_dicts(result.get("opLogRight", []), op_cls, target_cls),
            result.get("symbolMaps", {}))
