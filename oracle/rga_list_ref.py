"""RGA list-state restatement for the parity tests -- TEST INFRASTRUCTURE ONLY.

The reference's ``RGA`` (semmerge/crdt.py:23-57) holds its state in ``list``, a plain
``List[Elem]`` that callers may reorder, append to or reassign; every later event acts
on the list as it stands:
  insert(key, value)  before the first element, in list order, whose key tuple
                      (anchor, t, author, opid) is strictly greater (crdt.py:29-31, 48-57),
                      else at the end
  move(value, key)    drop the first live element with that value (crdt.py:33-37), then
                      insert(key, value)
  delete(value)       tombstone every element with that value (crdt.py:39-43)
This module keeps that state as [key tuple, value, tombstone] rows and applies the
events one at a time in pure Python (small cases only).  The GPU path (crdt.RGA) is
checked against it on lists in any order.
"""
from __future__ import annotations

from typing import Any, List, Sequence, Tuple

Row = List[Any]  # [key tuple, value, tombstone]


class ListRga:
    def __init__(self, rows: Sequence[Tuple[tuple, Any, bool]] = ()) -> None:
        self.rows: List[Row] = [[tuple(k), v, bool(tb)] for k, v, tb in rows]

    def _slot(self, key: tuple) -> int:
        # crdt.py:48-57: the first strictly greater key in the list's current order
        return next((i for i, r in enumerate(self.rows) if key < r[0]), len(self.rows))

    def insert(self, key: tuple, value: Any) -> None:
        self.rows.insert(self._slot(tuple(key)), [tuple(key), value, False])

    def move(self, value: Any, key: tuple) -> None:
        for i, r in enumerate(self.rows):  # crdt.py:33-37
            if not r[2] and r[1] == value:
                del self.rows[i]
                break
        self.insert(key, value)

    def delete(self, value: Any) -> None:
        for r in self.rows:  # crdt.py:39-43
            if r[1] == value:
                r[2] = True

    def state(self) -> List[Tuple[tuple, Any, bool]]:
        return [(r[0], r[1], r[2]) for r in self.rows]
