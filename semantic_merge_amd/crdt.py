"""Ordered-list CRDT (RGA) entry points, batched onto the GPU.

Reference: ``semmerge/crdt.py:8-57``.  ``Key``, ``Elem`` and the ``RGA`` method names and
argument meaning are unchanged; ``RGA`` records its event stream and
``materialize()`` replays it through ``smx_rga_replay`` (include/smx.h); ``RGA.list``
(the reference's state, crdt.py:26-27) replays it in the library's list mode, which
keeps the tombstoned elements.
:func:`replay` is the batched entry point: many independent lists in one launch.

Exact parallel restatement used by the device: the fate
of every element depends only on the events of its (list, value); survivors
are ordered by (key, creation order) because every insert keeps the list
sorted by key with equal keys in insertion order (``_find_insert_index``,
crdt.py:48-57, inserts before the first strictly greater key).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, List, Sequence, Tuple

import numpy as np

from .marshal import _EqClasses, _encode_ids

INSERT, MOVE, DELETE = 0, 1, 2


@dataclass(frozen=True)
class Key:
    """Position key (crdt.py:8-13); compared as the tuple (anchor, t, author, opid)."""

    anchor: str
    t: int
    author: str
    opid: str


@dataclass
class Elem:
    """List element (crdt.py:16-20)."""

    key: Key
    value: str
    tombstone: bool = False


Event = Tuple[int, Any, Any]  # (INSERT|MOVE|DELETE, key or None, value)


@dataclass
class RgaBatch:
    """Host image of ``smx_rga_ops``."""

    n_lists: int
    list_id: np.ndarray
    op: np.ndarray
    value: np.ndarray
    anchor: np.ndarray
    t: np.ndarray
    author: np.ndarray
    opid_hi: np.ndarray
    opid_lo: np.ndarray
    values: List[Any]          # event index -> value object (what materialize returns)

    @property
    def n(self) -> int:
        return len(self.op)


def _rank(xs: Sequence[Any]) -> np.ndarray:
    table = {x: i for i, x in enumerate(sorted(set(xs)))}
    return np.fromiter((table[x] for x in xs), np.uint32, len(xs))


def marshal_streams(streams: Sequence[Sequence[Event]]) -> RgaBatch:
    lids, ops, vals, anchors, ts, authors, opids, objs = [], [], [], [], [], [], [], []
    eq = _EqClasses()
    for lid, stream in enumerate(streams):
        for kind, key, value in stream:
            lids.append(lid)
            ops.append(kind)
            vals.append(eq(value))
            objs.append(value)
            if key is None:  # delete: key unused
                anchors.append("")
                ts.append(0)
                authors.append("")
                opids.append("")
            else:
                anchors.append(key.anchor)
                ts.append(key.t)
                authors.append(key.author)
                opids.append(key.opid)
    n = len(ops)
    tarr = np.fromiter(ts, np.int64, n) if all(
        type(x) is int and -2 ** 63 <= x < 2 ** 63 for x in ts) else _rank(ts).astype(np.int64)
    _, hi, lo = _encode_ids(opids) if n else (0, np.zeros(0, np.uint64), np.zeros(0, np.uint64))
    return RgaBatch(len(streams), np.asarray(lids, np.uint32), np.asarray(ops, np.uint8),
                    np.asarray(vals, np.uint32), _rank(anchors), tarr, _rank(authors),
                    hi, lo, objs)


def replay(streams: Sequence[Sequence[Event]]) -> List[List[Any]]:
    """Materialize every stream (one RGA per stream) on the GPU."""
    from ._lib import rga_replay_device  # the HIP library; raises if missing
    batch = marshal_streams(streams)
    _, src, offsets = rga_replay_device(batch)
    srcl = src.tolist()
    offl = offsets.tolist()
    return [[batch.values[s] for s in srcl[offl[i]:offl[i + 1]]] for i in range(len(streams))]


def replay_lists(streams: Sequence[Sequence[Event]]) -> List[List[Elem]]:
    """Every stream's final list state (crdt.py:26-27 ``RGA.list``) on the GPU: the
    elements in list order, tombstoned ones included, each as ``Elem(key, value,
    tombstone)`` with the key and value of the event that created it."""
    from ._lib import rga_replay_device  # the HIP library; raises if missing
    batch = marshal_streams(streams)
    _, src, offsets, tomb = rga_replay_device(batch, tombstones=True)
    events = [ev for stream in streams for ev in stream]
    srcl, tl, offl = src.tolist(), tomb.tolist(), offsets.tolist()
    return [[Elem(events[s][1], events[s][2], bool(tb)) for s, tb in
             zip(srcl[offl[i]:offl[i + 1]], tl[offl[i]:offl[i + 1]])] for i in range(len(streams))]


class RGA:
    """Drop-in for crdt.py:23-46: same methods; state is the recorded stream.  ``list``
    is the reference's ``List[Elem]`` state, computed on the GPU from the stream when it
    is read (a fresh list of fresh ``Elem`` objects each time: mutating it does not
    change the RGA, which is why it is read-only here)."""

    def __init__(self) -> None:
        self._events: List[Event] = []

    @property
    def list(self) -> List[Elem]:
        return replay_lists([self._events])[0]

    def insert(self, key: Key, value: str) -> None:
        self._events.append((INSERT, key, value))

    def move(self, value: str, key: Key) -> None:
        self._events.append((MOVE, key, value))

    def delete(self, value: str) -> None:
        self._events.append((DELETE, None, value))

    def materialize(self) -> List[str]:
        return replay([self._events])[0]
