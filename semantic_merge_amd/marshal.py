"""Host marshaler: two ``List[Op]`` -> the flat struct-of-arrays the device composes.

Every field is an exact, order- or equality-preserving image of what the
reference composer reads (``semmerge/compose.py``):

* ``kind``  u8   dense rank of ``precedence.get(op.type, 99)`` (compose.py:16-18,130-149)
* ``ts``    u64  order-preserving key of ``str(provenance.get("timestamp", default))``
                 compared by code point (compose.py:17)
* ``oid``   2xu64 order-preserving key of ``op.id`` (compose.py:18)
* ``sym``   u32  interned ``target.symbolId`` (dict membership / ``==``: compose.py:33,64)
* ``v0/v1`` i32  renames: equality class of ``params.get("newName")`` (the ``!=`` test,
                 compose.py:66) and the interned ``str(newName)`` (compose.py:72);
                 moves: interned ``str(newAddress)`` and ``str(newFile or file)`` or -1
                 (compose.py:75-82)

Key encodings (all exact; chosen once per call so every op uses the same one):

* timestamps: ISO-8601 ``YYYY-MM-DDTHH:MM:SS[.fff]Z`` packs to
  ``int(YYYYMMDDhhmmss) * 2000 + (2*fff | 1999)`` ('.' < 'Z' puts the
  fractional form first within a second); anything else -> dense rank of the
  unique strings in code-point order.
* ids: canonical lowercase UUID -> its 128-bit value (hex digits sort below
  'a'..'f' in both orders); ids of <= 15 UTF-8 bytes -> bytes zero padded plus
  a length byte (shorter prefix sorts first, as in Python); otherwise dense
  rank of the unique ids.
"""
from __future__ import annotations

from collections import OrderedDict

import re
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from .ops import KIND_MOVE, KIND_RENAME, KIND_RANK, KIND_UNKNOWN

DEFAULT_TIMESTAMP = "1970-01-01T00:00:00Z"  # compose.py:17
_ISO = re.compile(
    r"([0-9]{4})-([0-9]{2})-([0-9]{2})T([0-9]{2}):([0-9]{2}):([0-9]{2})(?:\.([0-9]{3}))?Z")
_UUID = re.compile(r"[0-9a-f]{8}-[0-9a-f]{4}-[0-9a-f]{4}-[0-9a-f]{4}-[0-9a-f]{12}")

TS_ISO, TS_RANK = 0, 1
ID_UUID, ID_PACKED, ID_RANK = 0, 1, 2


def iso_key(s: str):
    """Order-preserving u64 for the ISO forms lift.ts / Python produce, else None."""
    m = _ISO.fullmatch(s)
    if m is None:
        return None
    whole = int("".join(m.group(1, 2, 3, 4, 5, 6)))
    frac = m.group(7)
    return whole * 2000 + (2 * int(frac) if frac is not None else 1999)


def _utf8(s: str) -> bytes:
    # surrogatepass keeps code-point order for lone surrogates too.
    return s.encode("utf-8", "surrogatepass")


class _Tag:
    """Private tag so frozen containers never collide with user tuples."""

    __slots__ = ("name",)

    def __init__(self, name: str) -> None:
        self.name = name


_LIST, _DICT, _TUPLE = _Tag("list"), _Tag("dict"), _Tag("tuple")


def _freeze(v: Any):
    """Hashable stand-in with the same ``==`` behaviour as ``v``.

    ``bytearray`` compares equal to the ``bytes`` of the same content and ``set`` to
    the ``frozenset`` of the same elements, so they freeze to exactly those.  An
    ``OrderedDict`` compares order-sensitively with another one but not with a
    ``dict``, which no single key can express: it is rejected."""
    if isinstance(v, list):
        return (_LIST, tuple(_freeze(x) for x in v))
    if isinstance(v, OrderedDict):
        raise TypeError("OrderedDict")
    if isinstance(v, dict):
        return (_DICT, frozenset((k, _freeze(x)) for k, x in v.items()))
    if isinstance(v, bytearray):
        return bytes(v)
    if isinstance(v, set):
        return frozenset(v)
    if isinstance(v, tuple):
        try:
            hash(v)
            return v
        except TypeError:
            return (_TUPLE, tuple(_freeze(x) for x in v))
    hash(v)  # raises TypeError for anything we cannot reason about
    return v


def eq_key(v: Any):
    """Hashable key of a non-scalar newName with ``==`` semantics (``_freeze``)."""
    try:
        return _freeze(v)
    except TypeError as exc:
        raise TypeError(f"newName of type {type(v).__name__} is not comparable "
                        "by the device composer") from exc


class _EqClasses:
    """Interns values by Python ``==`` (the ``!=`` test of compose.py:66)."""

    def __init__(self) -> None:
        self._ids: Dict[Any, int] = {}
        self._next = 0

    def __call__(self, v: Any) -> int:
        if isinstance(v, float) and v != v:  # NaN != NaN, even the same object
            self._next += 1
            return self._next - 1
        key = v if isinstance(v, (str, int, float, type(None))) else eq_key(v)
        got = self._ids.get(key)
        if got is None:
            got = self._ids[key] = self._next
            self._next += 1
        return got


@dataclass
class SoA:
    """Host image of ``smx_ops`` (include/smx.h)."""

    n_a: int
    n_b: int
    kind: np.ndarray      # u8
    ts: np.ndarray        # u64
    oid_hi: np.ndarray    # u64
    oid_lo: np.ndarray    # u64
    sym: np.ndarray       # u32
    v0: np.ndarray        # i32
    v1: np.ndarray        # i32
    n_sym: int
    strings: List[str] = field(default_factory=list)   # string table for v-ids
    ts_mode: int = TS_ISO
    id_mode: int = ID_UUID

    @property
    def n(self) -> int:
        return self.n_a + self.n_b


def _encode_ts(ts_strings: Sequence[str]):
    uniq = dict.fromkeys(ts_strings)
    keys = {}
    for s in uniq:
        k = iso_key(s)
        if k is None:
            break
        keys[s] = k
    else:
        return TS_ISO, np.fromiter((keys[s] for s in ts_strings), np.uint64, len(ts_strings))
    ranks = {s: i for i, s in enumerate(sorted(uniq))}
    return TS_RANK, np.fromiter((ranks[s] for s in ts_strings), np.uint64, len(ts_strings))


def _encode_ids(ids: Sequence[Any]):
    n = len(ids)
    hi = np.empty(n, np.uint64)
    lo = np.empty(n, np.uint64)
    if all(type(i) is str and _UUID.fullmatch(i) for i in ids):
        for k, s in enumerate(ids):
            v = int(s.replace("-", ""), 16)
            hi[k] = v >> 64
            lo[k] = v & 0xFFFFFFFFFFFFFFFF
        return ID_UUID, hi, lo
    if all(isinstance(i, str) for i in ids):
        enc = [_utf8(s) for s in ids]
        if all(len(b) <= 15 for b in enc):
            for k, b in enumerate(enc):
                padded = b.ljust(15, b"\0") + bytes([len(b)])
                hi[k] = int.from_bytes(padded[:8], "big")
                lo[k] = int.from_bytes(padded[8:], "big")
            return ID_PACKED, hi, lo
    ranks = {s: i for i, s in enumerate(sorted(set(ids)))}
    hi[:] = 0
    for k, s in enumerate(ids):
        lo[k] = ranks[s]
    return ID_RANK, hi, lo


def marshal(delta_a: Sequence[Any], delta_b: Sequence[Any]) -> SoA:
    """Build the SoA for ``compose_oplogs(delta_a, delta_b)``; A ops first."""
    ops = list(delta_a) + list(delta_b)
    n = len(ops)
    kind = np.empty(n, np.uint8)
    sym = np.empty(n, np.uint32)
    v0 = np.full(n, -1, np.int32)
    v1 = np.full(n, -1, np.int32)
    ts_str: List[str] = [""] * n
    ids: List[Any] = [None] * n

    syms: Dict[Any, int] = {}
    strings: Dict[str, int] = {}
    eq = _EqClasses()

    def sid(s: str) -> int:
        got = strings.get(s)
        if got is None:
            got = strings[s] = len(strings)
        return got

    for k, op in enumerate(ops):
        kr = KIND_RANK.get(op.type, KIND_UNKNOWN)   # precedence.get(type, 99)
        kind[k] = kr
        ts_str[k] = str(op.provenance.get("timestamp", DEFAULT_TIMESTAMP))
        ids[k] = op.id
        s = op.target.symbolId
        got = syms.get(s)
        if got is None:
            got = syms[s] = len(syms)
        sym[k] = got
        params = op.params
        if kr == KIND_RENAME:
            name = params.get("newName")
            v0[k] = eq(name)
            v1[k] = sid(str(name))
        elif kr == KIND_MOVE:
            addr = params.get("newAddress")
            if addr is not None:
                v0[k] = sid(str(addr))
            nfile = params.get("newFile") or params.get("file")
            if nfile is not None:
                v1[k] = sid(str(nfile))
    ts_mode, ts = _encode_ts(ts_str)
    id_mode, hi, lo = _encode_ids(ids)
    return SoA(len(delta_a), len(delta_b), kind, ts, hi, lo, sym, v0, v1, max(len(syms), 1),
               list(strings), ts_mode, id_mode)


def marshal_native(delta_a: Sequence[Any], delta_b: Sequence[Any], cols: Optional[dict] = None) -> SoA:
    """``marshal`` done by the native host module (csrc/smx_host.cpp): same SoA, same
    exceptions.  Only non-ISO timestamps and ids that are neither canonical UUIDs nor
    short strings go back to the Python encoders above (dense ranks need a sort).
    cols: preallocated output columns (kind, ts, oid_hi, oid_lo, sym, v0, v1 of n ops,
    e.g. ComposeSession.staging's pinned views)."""
    from ._host import host
    ops = list(delta_a) + list(delta_b)
    n = len(ops)
    if cols is None:
        kind, ts, hi, lo = np.empty(n, np.uint8), np.empty(n, np.uint64), np.empty(n, np.uint64), np.empty(n, np.uint64)
        sym, v0, v1 = np.empty(n, np.uint32), np.empty(n, np.int32), np.empty(n, np.int32)
    else:
        kind, ts, hi, lo, sym, v0, v1 = (cols[k] for k in ("kind", "ts", "oid_hi", "oid_lo", "sym", "v0", "v1"))
    n_sym, strings, ts_ok, id_mode, ts_str, ids = host().marshal_ops(
        ops, KIND_RANK, KIND_UNKNOWN, KIND_MOVE, KIND_RENAME, DEFAULT_TIMESTAMP, eq_key,
        kind, ts, hi, lo, sym, v0, v1)
    ts_mode = TS_ISO
    if not ts_ok:
        ts_mode, ts = _encode_ts(ts_str)
    if id_mode < 0:
        id_mode, hi, lo = _encode_ids(ids)
    return SoA(len(delta_a), len(delta_b), kind, ts, hi, lo, sym, v0, v1, max(n_sym, 1),
               strings, ts_mode, id_mode)
