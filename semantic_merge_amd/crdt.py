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
    _, src, offsets = rga_replay_device(batch, grouped=True)  # (marshal_streams: stream after stream)
    srcl = src.tolist()
    offl = offsets.tolist()
    return [[batch.values[s] for s in srcl[offl[i]:offl[i + 1]]] for i in range(len(streams))]


def replay_lists(streams: Sequence[Sequence[Event]]) -> List[List[Elem]]:
    """Every stream's final list state (crdt.py:26-27 ``RGA.list``) on the GPU: the
    elements in list order, tombstoned ones included, each as ``Elem(key, value,
    tombstone)`` with the key and value of the event that created it."""
    from ._lib import rga_replay_device  # the HIP library; raises if missing
    batch = marshal_streams(streams)
    _, src, offsets, tomb = rga_replay_device(batch, tombstones=True, grouped=True)
    events = [ev for stream in streams for ev in stream]
    srcl, tl, offl = src.tolist(), tomb.tolist(), offsets.tolist()
    return [[Elem(events[s][1], events[s][2], bool(tb)) for s, tb in
             zip(srcl[offl[i]:offl[i + 1]], tl[offl[i]:offl[i + 1]])] for i in range(len(streams))]


class RGA:
    """Drop-in for crdt.py:23-46: same methods, and ``list`` (crdt.py:26-27) is the
    reference's mutable ``List[Elem]`` state.

    Events are recorded and replayed on the GPU (``smx_rga_replay``) when the state is
    needed.  Reading ``list`` folds the pending events into the state and returns the
    SAME list object on every read, before and after new events, so
    ``rga.list.append(e)`` or ``rga.list[0].tombstone = True`` change the RGA as they do in
    the reference; assigning ``rga.list = L`` makes ``L`` the state, and later events are
    folded into ``L`` itself.  (The reference mutates the object at each call; here a
    held reference sees the events at the next fold: the next read of ``list`` or
    ``materialize()``.)  A later fold replays the state as
    a prefix of the stream (each live element as its insert; each tombstoned one as an
    insert of a private value that is then deleted, so no later event can touch it) and
    keeps the existing ``Elem`` objects: a later ``delete`` sets ``tombstone`` on them in
    place, as crdt.py:40-43 does.  A state the caller put out of key order replays with
    each element keyed by the running maximum of the keys before it (``_effective_keys``):
    the same insert slots as crdt.py:48-57's scan of the list as it stands."""

    def __init__(self) -> None:
        self._events: List[Event] = []
        self._list: "List[Elem] | None" = None  # the state, once read or assigned

    @property
    def list(self) -> List[Elem]:
        if self._list is None or self._events:
            out = self._fold()
            if self._list is None:
                self._list = out
            else:  # the caller's list object is the state (crdt.py:27, 31, 36): fold into it
                self._list[:] = out
            self._events = []
        return self._list

    @list.setter
    def list(self, value: List[Elem]) -> None:
        self._list = value
        self._events = []

    def _fold(self) -> List[Elem]:
        base = self._list or []
        if not base:
            return replay_lists([self._events])[0]
        events = self._events
        while True:
            eff, ordered = _effective_keys(base)
            j = -1 if ordered else next((i for i, ev in enumerate(events) if ev[0] == MOVE), -1)
            if j < 0:
                return _replay_onto(base, eff, events)
            # A list out of key order whose events hold a move: the move's pop can lower
            # the effective keys after it, so the events are replayed up to it, then its pop
            # alone (its insert dropped), and its insert opens the next round on the new list.
            if j:
                base = _replay_onto(base, eff, events[:j])
                eff, _ = _effective_keys(base)
            _, key, value = events[j]
            base = _replay_onto(base, eff, [events[j]], drop_new=True)
            events = [(INSERT, key, value)] + list(events[j + 1:])
    def insert(self, key: Key, value: str) -> None:
        self._events.append((INSERT, key, value))

    def move(self, value: str, key: Key) -> None:
        self._events.append((MOVE, key, value))

    def delete(self, value: str) -> None:
        self._events.append((DELETE, None, value))

    def materialize(self) -> List[str]:
        if self._list is None:
            return replay([self._events])[0]
        return [e.value for e in self.list if not e.tombstone]


def _effective_keys(base: Sequence[Elem]) -> Tuple[List[Key], bool]:
    """Each element's insert key for the replay of a list state, and whether the list is
    in key order.  An insert goes before the first element, in list order, whose key is
    strictly greater (crdt.py:48-57): the first element whose running maximum of keys
    is greater.  So the state replays as inserts keyed by that running maximum -- the
    list's own keys when it is in key order (what insert() and move() keep); the
    running maximum makes a caller-reordered list a key-ordered one with the same
    insert slots, and a new element's maximum is its own key.  Inserts and deletes leave
    the other elements' maxima unchanged; a move's pop may lower them (RGA._fold)."""
    eff: List[Key] = []
    ordered = True
    top = None
    for e in base:
        k = (e.key.anchor, e.key.t, e.key.author, e.key.opid)
        if top is None or k >= top:
            top = k
            eff.append(e.key)
        else:  # (below the running maximum: inserts see the maximum here)
            ordered = False
            eff.append(eff[-1])
    return eff, ordered


def _replay_onto(base: Sequence[Elem], eff: Sequence[Key], events: Sequence[Event],
                 drop_new: bool = False) -> List[Elem]:
    """The list state `base` (insert keys `eff`) followed by `events`, replayed on the
    GPU.  Each live element replays as its insert, each tombstoned one as an insert of
    a private value that is then deleted (no later event can touch it); the existing
    Elem objects are kept (a delete tombstones them in place, crdt.py:40-43), every
    event-created element is a new Elem.  drop_new: leave the event-created elements
    out (a move's pop replayed alone)."""
    stream: List[Event] = []
    origin: List[int] = []  # stream index -> base index (-1: a later event)
    for i, e in enumerate(base):
        if e.tombstone:
            tag = object()  # equal to nothing else: no later move/delete reaches it
            stream.append((INSERT, eff[i], tag))
            stream.append((DELETE, None, tag))
            origin += [i, -1]
        else:
            stream.append((INSERT, eff[i], e.value))
            origin.append(i)
    nb = len(stream)
    stream += list(events)
    src, tomb = _replay_list_src(stream)
    out: List[Elem] = []
    for s, tb in zip(src, tomb):
        if s < nb:
            e = base[origin[s]]
            if tb:
                e.tombstone = True
        elif drop_new:
            continue
        else:
            _, key, value = stream[s]
            e = Elem(key, value, bool(tb))
        out.append(e)
    return out


def _replay_list_src(stream: Sequence[Event]) -> Tuple[List[int], List[int]]:
    """One stream in list mode on the GPU: (creating event index, tombstone) per element
    of the final list, in list order."""
    from ._lib import rga_replay_device  # the HIP library; raises if missing
    batch = marshal_streams([stream])
    _, src, offsets, tomb = rga_replay_device(batch, tombstones=True, grouped=True)
    n = int(offsets[1])
    return src[:n].tolist(), tomb[:n].tolist()
