"""Op-log decoding on the native host module: the data format on
the input side of compose.

* ``ops_from_dicts(items)`` is ``[Op.from_dict(d) for d in items]``
  (``semmerge/ops.py:89-100``): same coercions, same evaluation order, same exceptions.
  It runs in ``csrc/smx_host.cpp``. Plain dataclasses (the reference's ``Op`` and
  ``Target``) are built as their generated ``__init__`` would build them; any other
  class is called.
* ``OpLog`` restates ``semmerge/ops.py:106-121``: ``to_json`` / ``from_json`` with
  orjson's semantics (compact output, non-ASCII kept, NaN / Infinity written as null
  and rejected on input, non-string keys and integers beyond 64 bits rejected) --
  orjson itself when it is importable, the standard json module held to those rules
  when it is not; ``from_json`` decodes through ``ops_from_dicts``.
* ``oplog_from_json(text)`` is ``OpLog.from_json(text).ops``.
* ``ops_from_worker_result(result)`` is what ``TSWorker.build_and_diff`` does with the
  worker's JSON-RPC result (``semmerge/lang/ts/bridge.py:36-40``).

Pass the reference's own classes as ``op_cls`` / ``target_cls`` to get its ``Op``
objects back.
"""
from __future__ import annotations

import json
import math
from dataclasses import dataclass, field
from typing import Any, Dict, Iterable, List, Sequence, Tuple

from ._host import host
from .materialize import smx_host_ctor_mode
from .ops import Op, Target


def ops_from_dicts(items: Sequence[Any], op_cls: type = Op, target_cls: type = Target) -> List[Any]:
    return host().ops_from_dicts(list(items), op_cls, target_cls, smx_host_ctor_mode)


def _orjson():
    try:
        import orjson
        return orjson
    except ImportError:
        return None


def _json_ready(x: Any) -> Any:
    """orjson's output rules on the standard encoder: non-finite floats -> null,
    string keys only, integers within 64 bits."""
    if isinstance(x, float):
        return x if math.isfinite(x) else None
    if isinstance(x, bool) or x is None or isinstance(x, str):
        return x
    if isinstance(x, int):
        if not -(2 ** 63) <= x < 2 ** 64:
            raise TypeError("Integer exceeds 64-bit range")
        return x
    if isinstance(x, dict):
        out = {}
        for k, v in x.items():
            if not isinstance(k, str):
                raise TypeError("Dict key must be str")
            out[k] = _json_ready(v)
        return out
    if isinstance(x, (list, tuple)):
        return [_json_ready(v) for v in x]
    raise TypeError(f"Type is not JSON serializable: {type(x).__name__}")


def dumps(obj: Any) -> str:
    """``orjson.dumps(obj).decode()`` (ops.py:113)."""
    oj = _orjson()
    if oj is not None:
        return oj.dumps(obj).decode()
    return json.dumps(_json_ready(obj), separators=(",", ":"), ensure_ascii=False)


def _reject_constant(name: str):
    raise json.JSONDecodeError(f"unexpected {name}", name, 0)


def loads(data: Any) -> Any:
    """``orjson.loads(data)`` (ops.py:117): str or bytes, NaN / Infinity rejected."""
    oj = _orjson()
    if oj is not None:
        return oj.loads(data)
    if isinstance(data, (bytes, bytearray, memoryview)):
        data = bytes(data).decode("utf-8")
    return json.loads(data, parse_constant=_reject_constant)


@dataclass
class OpLog:
    """Collection of operations (ops.py:106-121)."""

    ops: List[Any] = field(default_factory=list)

    def to_json(self) -> str:
        return dumps([o.to_dict() for o in self.ops])

    @staticmethod
    def from_json(data: Any, op_cls: type = Op, target_cls: type = Target) -> "OpLog":
        return OpLog(ops_from_dicts(loads(data), op_cls, target_cls))

    def extend(self, ops: Iterable[Any]) -> None:
        self.ops.extend(ops)


def oplog_from_json(data: Any, op_cls: type = Op, target_cls: type = Target) -> List[Any]:
    return OpLog.from_json(data, op_cls, target_cls).ops


def ops_from_worker_result(result: Dict[str, Any], op_cls: type = Op,
                           target_cls: type = Target) -> Tuple[List[Any], List[Any], Any]:
    """(opLogLeft ops, opLogRight ops, symbolMaps) of a ``buildAndDiff`` result."""
    return (ops_from_dicts(result.get("opLogLeft", []), op_cls, target_cls),
            ops_from_dicts(result.get("opLogRight", []), op_cls, target_cls),
            result.get("symbolMaps", {}))
