"""Pure-Python restatement of the reference composer on the SoA, for TESTS ONLY.

Test infrastructure like oracle/compose_ref.c (same steps, same outputs): it is the
single-core Python leg of bench.py's cpu_baseline and is checked against the C
oracle in tests/test_oracle_py.py.  It walks /root/reference/semmerge/compose.py:
  sort_key / sorted       compose.py:16-21  (stable per-branch sort on the SoA keys)
  merge loop              compose.py:51-112 (A on ties, compose.py:54)
  DivergentRename skip    compose.py:60-70, 88-98
  rename / move chains    compose.py:71-82, 99-110
  materialize             compose.py:30-49 (as the string ids the SoA output holds)
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

MOVE, RENAME, NONE = 0, 1, -1


def compose(soa) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
    """(order, addr, file, ctx, conflict_pairs[n, 2]) of one merge, like oracle.compose."""
    na, nb = soa.n_a, soa.n_b
    kind = soa.kind.tolist()
    ts = soa.ts.tolist()
    hi = soa.oid_hi.tolist()
    lo = soa.oid_lo.tolist()
    sym = soa.sym.tolist()
    v0 = soa.v0.tolist()
    v1 = soa.v1.tolist()

    def key(i):
        return (kind[i], ts[i], hi[i], lo[i])

    ops_a = sorted(range(na), key=key)               # stable: index breaks ties
    ops_b = sorted(range(na, na + nb), key=key)
    rename_chain: dict = {}
    move_addr: dict = {}
    move_file: dict = {}
    order: List[int] = []
    addr: List[int] = []
    file: List[int] = []
    ctx: List[int] = []
    conflicts: List[Tuple[int, int]] = []
    ia = ib = 0
    while ia < na or ib < nb:
        if ia < na and ib < nb:
            a, b = ops_a[ia], ops_b[ib]
            if kind[a] == RENAME and kind[b] == RENAME and sym[a] == sym[b] and v0[a] != v0[b]:
                conflicts.append((a, b))
                ia += 1
                ib += 1
                continue
            use_a = key(a) <= key(b)
        else:
            use_a = ia < na
        if use_a:
            i = ops_a[ia]
            ia += 1
        else:
            i = ops_b[ib]
            ib += 1
        s = sym[i]
        if kind[i] == RENAME:
            rename_chain[s] = v1[i]
        elif kind[i] == MOVE:
            if v0[i] != NONE:
                move_addr[s] = v0[i]
            if v1[i] != NONE:
                move_file[s] = v1[i]
        order.append(i)
        addr.append(move_addr.get(s, NONE))
        file.append(move_file.get(s, NONE))
        ctx.append(rename_chain.get(s, NONE) if kind[i] != RENAME else NONE)
    i32 = np.int32
    pairs = np.array(conflicts, dtype=i32).reshape(-1, 2)
    return (np.array(order, i32), np.array(addr, i32), np.array(file, i32), np.array(ctx, i32), pairs)
