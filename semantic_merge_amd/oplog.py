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
* ``decode_pair(text_a, text_b)`` is both ``OpLog.from_json`` calls plus the compose SoA
  of their ops (``marshal.marshal_native``) in one native pass over the texts
  (the wire format straight into SoA); ``compose_json`` runs the
  drop-in compose on it.
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


def _utf8_str(x: str) -> str:
    """orjson.dumps refuses str with lone surrogates (not UTF-8)."""
    try:
        x.encode("utf-8")
    except UnicodeEncodeError:
        raise TypeError("str is not valid UTF-8: surrogates not allowed") from None
    return x


def _json_ready(x: Any) -> Any:
    """orjson's output rules on the standard encoder: non-finite floats -> null,
    string keys only, integers within 64 bits, str without lone surrogates."""
    if isinstance(x, float):
        return x if math.isfinite(x) else None
    if isinstance(x, str):
        return _utf8_str(x)
    if isinstance(x, bool) or x is None:
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
            out[_utf8_str(k)] = _json_ready(v)
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


def loads(data: Any) -> Any:
    """``orjson.loads(data)`` (ops.py:117): str or bytes; NaN / Infinity, lone
    surrogates (in the text or as escapes) and invalid UTF-8 rejected with
    json.JSONDecodeError (orjson.JSONDecodeError subclasses it).  Without orjson: the
    native strict reader (csrc/smx_host.cpp JsonReader; the json module's results)."""
    oj = _orjson()
    if oj is not None:
        return oj.loads(data)
    if isinstance(data, str):
        try:
            data.encode("utf-8")
        except UnicodeEncodeError:
            raise json.JSONDecodeError("str is not valid UTF-8: surrogates not allowed", data, 0) from None
    return host().json_loads(data)


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


def decode_pair(text_a: Any, text_b: Any, op_cls: type = Op, target_cls: type = Target):
    """(ops_a, ops_b, soa): ``OpLog.from_json`` of both branch logs and the compose SoA
    of ``ops_a + ops_b`` (equal to ``marshal_native(ops_a, ops_b)``), in one pass."""
    import numpy as np
    from .marshal import (DEFAULT_TIMESTAMP, SoA, TS_ISO, _encode_ids, _encode_ts, eq_key)
    from .ops import KIND_MOVE, KIND_RANK, KIND_RENAME, KIND_UNKNOWN
    if _orjson() is not None:  # orjson's own reader decides what parses
        from .marshal import marshal_native
        ops_a = OpLog.from_json(text_a, op_cls, target_cls).ops
        ops_b = OpLog.from_json(text_b, op_cls, target_cls).ops
        return ops_a, ops_b, marshal_native(ops_a, ops_b)
    (ops_a, ops_b), summ, kind, ts, hi, lo, sym, v0, v1 = host().decode_oplogs(
        (text_a, text_b), op_cls, target_cls, smx_host_ctor_mode, KIND_RANK, KIND_UNKNOWN, KIND_MOVE,
        KIND_RENAME, DEFAULT_TIMESTAMP, eq_key)
    n_sym, strings, ts_ok, id_mode, ts_str, ids = summ
    kind = np.frombuffer(kind, np.uint8)
    ts = np.frombuffer(ts, np.uint64)
    hi, lo = np.frombuffer(hi, np.uint64), np.frombuffer(lo, np.uint64)
    ts_mode = TS_ISO
    if not ts_ok:
        ts_mode, ts = _encode_ts(ts_str)
    if id_mode < 0:
        id_mode, hi, lo = _encode_ids(ids)
    soa = SoA(len(ops_a), len(ops_b), kind, ts, hi, lo, np.frombuffer(sym, np.uint32),
              np.frombuffer(v0, np.int32), np.frombuffer(v1, np.int32), max(n_sym, 1), strings, ts_mode,
              id_mode)
    return ops_a, ops_b, soa


def compose_json(text_a: Any, text_b: Any, op_cls: type = Op, target_cls: type = Target):
    """compose_oplogs(OpLog.from_json(text_a).ops, OpLog.from_json(text_b).ops) with the
    decode and the marshal fused (decode_pair)."""
    from ._lib import dropin_session
    from .materialize import materialize_conflicts, materialize_ops_native
    ops_a, ops_b, soa = decode_pair(text_a, text_b, op_cls, target_cls)
    with dropin_session() as sess:  # (views of its staging area, materialised while held)
        order, addr, file, ctx, pairs = sess.compose(soa, copy=False)
        ops = ops_a + ops_b
        return materialize_ops_native(ops, soa.kind, soa.strings, order, addr, file, ctx), \
            materialize_conflicts(ops, pairs)


def ops_from_worker_result(result: Dict[str, Any], op_cls: type = Op,
                           target_cls: type = Target) -> Tuple[List[Any], List[Any], Any]:
    """(opLogLeft ops, opLogRight ops, symbolMaps) of a ``buildAndDiff`` result."""
    return (ops_from_dicts(result.get("opLogLeft", []), op_cls, target_cls),
            ops_from_dicts(result.get("opLogRight", []), op_cls, target_cls),
            result.get("symbolMaps", {}))
