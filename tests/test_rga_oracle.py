"""The CPU RGA oracle (oracle/crdt_ref.c) reproduces the reference RGA's outputs."""
from oracle import oracle
from semantic_merge_amd.crdt import DELETE, INSERT, MOVE, Key, marshal_streams

from _util import load

OPS = {"insert": INSERT, "move": MOVE, "delete": DELETE}


def to_streams(cases):
    streams = []
    for case in cases:
        s = []
        for ev in case["events"]:
            if ev[0] == "delete":
                s.append((DELETE, None, ev[1]))
            else:
                s.append((OPS[ev[0]], Key(*ev[2]), ev[1]))
        streams.append(s)
    return streams


def test_rga_oracle_matches_reference():
    cases = load("rga_cases.json")
    b = marshal_streams(to_streams(cases))
    vals, src, offs = oracle.rga(b.n_lists, b.list_id, b.op, b.value, b.anchor, b.t,
                                 b.author, b.opid_hi, b.opid_lo)
    srcl, offl = src.tolist(), offs.tolist()
    for i, case in enumerate(cases):
        got = [b.values[s] for s in srcl[offl[i]:offl[i + 1]]]
        assert got == case["out"], f"rga case {i}"


def _list_ref_script(steps):
    """tools/make_golden.py's RGA mutation scripts on oracle/rga_list_ref.py."""
    from oracle.rga_list_ref import ListRga
    r, held, rec, unordered = ListRga(), None, [], 0
    for st in steps:
        op = st[0]
        if op == "insert":
            r.insert(tuple(st[2]), st[1])
        elif op == "move":
            r.move(st[1], tuple(st[2]))
        elif op == "delete":
            r.delete(st[1])
        elif op == "read":
            rec.append([[list(k), v, tb] for k, v, tb in r.state()])
            ks = [row[0] for row in r.rows]
            unordered += any(b < a for a, b in zip(ks, ks[1:]))
        elif op == "materialize":
            rec.append([v for _, v, tb in r.state() if not tb])
        elif op == "append":
            r.rows.append([tuple(st[1]), st[2], st[3]])
        elif op == "pop":
            r.rows.pop(st[1])
        elif op == "set_tomb":
            r.rows[st[1]][2] = st[2]
        elif op == "assign":
            r.rows = [[tuple(k), v, tb] for k, v, tb in st[1]]
        elif op == "hold":
            held = r.rows[st[1]]
        elif op == "held":
            rec.append(None if held is None else held[2])
    return rec, unordered


def test_list_ref_matches_reference_mutation_scripts():
    """oracle/rga_list_ref.py (the list-state checker of the GPU RGA class) reproduces
    the reference RGA's results on the 300 mutation scripts (appends, pops, tombstone
    flips, assignments, held elements).  Those scripts keep their lists in key order, so
    for states out of key order the checker rests on its line-by-line restatement of
    crdt.py:29-57 (no reference output covers them)."""
    for i, case in enumerate(load("rga_mutation_cases.json")):
        rec, _ = _list_ref_script(case["steps"])
        assert rec == case["out"], f"mutation script {i}"


def test_effective_keys_give_the_scan_slot():
    """crdt._effective_keys: on a list in any order, the slot of crdt.py:48-57's scan
    (before the first strictly greater key) is the upper bound of the new key among
    the running-maximum keys -- the slot the device replay of a key-ordered list takes."""
    import bisect
    import random
    from semantic_merge_amd.crdt import Elem, _effective_keys
    rnd = random.Random(5)
    tup = lambda k: (k.anchor, k.t, k.author, k.opid)
    for _ in range(500):
        base = [Elem(Key(rnd.choice("abc"), rnd.randrange(3), "u", "o"), "v") for _ in range(rnd.randrange(8))]
        eff, ordered = _effective_keys(base)
        ks = [tup(e.key) for e in base]
        assert ordered == all(a <= b for a, b in zip(ks, ks[1:]))
        assert [tup(k) for k in eff] == sorted(tup(k) for k in eff)  # non-decreasing
        for _ in range(5):
            k = (rnd.choice("abcd"), rnd.randrange(4), "u", "o")
            scan = next((i for i, x in enumerate(ks) if k < x), len(ks))
            assert scan == bisect.bisect_right([tup(x) for x in eff], k)
