"""GPU parity for the batched RGA replay (crdt.py:23-57) through the C ABI."""
import numpy as np
import pytest

from oracle import oracle
from semantic_merge_amd import synth
from semantic_merge_amd._lib import rga_replay_device
from semantic_merge_amd.crdt import RGA, Elem, Key, marshal_streams, replay, replay_lists

from _util import load
from test_rga_oracle import to_streams

pytestmark = pytest.mark.gpu


def test_rga_golden_cases_gpu():
    cases = load("rga_cases.json")
    got = replay(to_streams(cases))
    for i, case in enumerate(cases):
        assert got[i] == case["out"], f"rga case {i}"


def test_rga_class_dropin():
    r = RGA()
    r.insert(Key("root", 1, "u1", "o1"), "a")
    r.insert(Key("root", 0, "u1", "o2"), "b")
    r.move("a", Key("root", -1, "u2", "o3"))
    r.insert(Key("root", 5, "u1", "o4"), "c")
    r.delete("b")
    assert r.materialize() == ["a", "c"]


def test_rga_list_state_golden_gpu():
    """RGA.list (crdt.py:26-27) in the library's list mode: every element in list order,
    tombstoned ones included, equals the reference's list after each golden stream
    (tests/golden/rga_list_cases.json, tools/make_golden.py --only rga_list)."""
    cases = load("rga_cases.json")
    want = load("rga_list_cases.json")
    got = replay_lists(to_streams(cases))
    assert sum(e[2] for w in want for e in w) > 100  # tombstones present
    for i, (g, w) in enumerate(zip(got, want)):
        assert [[[e.key.anchor, e.key.t, e.key.author, e.key.opid], e.value, e.tombstone] for e in g] == w, \
            f"rga list case {i}"


def test_rga_class_list_property():
    r = RGA()
    r.insert(Key("root", 1, "u1", "o1"), "a")
    r.insert(Key("root", 0, "u1", "o2"), "b")
    r.move("a", Key("root", -1, "u2", "o3"))
    r.delete("b")
    assert r.list == [Elem(Key("root", -1, "u2", "o3"), "a", False), Elem(Key("root", 0, "u1", "o2"), "b", True)]
    assert [e.value for e in r.list if not e.tombstone] == r.materialize() == ["a"]


def _run_mutation_script(steps):
    r, held, rec = RGA(), None, []

    def snap():
        return [[[e.key.anchor, e.key.t, e.key.author, e.key.opid], e.value, e.tombstone] for e in r.list]

    for st in steps:
        op = st[0]
        if op == "insert":
            r.insert(Key(*st[2]), st[1])
        elif op == "move":
            r.move(st[1], Key(*st[2]))
        elif op == "delete":
            r.delete(st[1])
        elif op == "read":
            rec.append(snap())
        elif op == "materialize":
            rec.append(r.materialize())
        elif op == "append":
            r.list.append(Elem(Key(*st[1]), st[2], st[3]))
        elif op == "pop":
            r.list.pop(st[1])
        elif op == "set_tomb":
            r.list[st[1]].tombstone = st[2]
        elif op == "assign":
            r.list = [Elem(Key(*k), v, tb) for k, v, tb in st[1]]
        elif op == "hold":
            held = r.list[st[1]]
        elif op == "held":
            rec.append(None if held is None else held.tombstone)
    return rec


def test_rga_list_mutable_state_golden_gpu():
    """RGA.list is the reference's mutable attribute (crdt.py:26-27): reads return the
    state object itself, appends / pops / tombstone flips / assignments change the RGA,
    and an element held across a later delete() is tombstoned in place (crdt.py:40-43).
    300 scripts, the reference's own results (tools/make_golden.py --only rga_mut)."""
    cases = load("rga_mutation_cases.json")
    assert sum(1 for c in cases for s in c["steps"] if s[0] in ("append", "pop", "set_tomb", "assign")) > 100
    for i, case in enumerate(cases):
        assert _run_mutation_script(case["steps"]) == case["out"], f"rga mutation script {i}"


def test_rga_list_object_held_across_events():
    """The list object is the state (crdt.py:27): a reference held before insert / move /
    delete, or a list the caller assigned, is the object the later events are folded into
    (each Elem created by an event is new, base Elems are kept and tombstoned in place).
    Expected states: the reference's own RGA on the same calls (checked in the build
    container)."""
    r = RGA()
    r.insert(Key("root", 1, "u1", "o1"), "a")
    lst = r.list
    held = lst[0]
    r.insert(Key("root", 0, "u1", "o2"), "b")
    r.move("a", Key("root", 2, "u2", "o3"))
    r.delete("b")
    assert r.materialize() == ["a"]
    assert r.list is lst
    assert lst == [Elem(Key("root", 0, "u1", "o2"), "b", True), Elem(Key("root", 2, "u2", "o3"), "a", False)]
    assert all(e is not held for e in lst)  # the moved element was popped (crdt.py:36)
    L = [Elem(Key("a", 0, "u", "o1"), "x"), Elem(Key("c", 0, "u", "o2"), "y")]
    r.list = L
    x = L[0]
    r.insert(Key("b", 0, "u", "o3"), "z")
    r.delete("x")
    assert r.list is L
    assert L == [Elem(Key("a", 0, "u", "o1"), "x", True), Elem(Key("b", 0, "u", "o3"), "z"),
                 Elem(Key("c", 0, "u", "o2"), "y")]
    assert L[0] is x and x.tombstone  # tombstoned in place (crdt.py:40-43)


def _out_of_order_script(rng, n_steps):
    """A random script over a caller-reordered list: assignments of shuffled lists,
    out-of-order appends, reversals, and inserts / moves / deletes with duplicate keys
    and values."""
    keys = [(a, t, u, o) for a in "abc" for t in range(2) for u in ("u1", "u2") for o in ("o1",)]
    vals = ["v%d" % i for i in range(5)]
    steps = []
    for _ in range(n_steps):
        r = rng.random()
        k = list(keys[rng.integers(len(keys))])
        v = vals[rng.integers(len(vals))]
        if r < 0.08:
            m = int(rng.integers(0, 7))
            steps.append(("assign", [(list(keys[rng.integers(len(keys))]), vals[rng.integers(len(vals))],
                                      bool(rng.random() < 0.2)) for _ in range(m)]))
        elif r < 0.16:
            steps.append(("append", k, v, bool(rng.random() < 0.2)))
        elif r < 0.2:
            steps.append(("reverse",))
        elif r < 0.5:
            steps.append(("insert", v, k))
        elif r < 0.7:
            steps.append(("move", v, k))
        elif r < 0.8:
            steps.append(("delete", v))
        else:
            steps.append(("read",))
    steps.append(("read",))
    return steps


def test_rga_list_out_of_key_order_matches_reference_semantics():
    """A list the caller put out of key order (assigned, appended to, reversed): later
    inserts go before the first greater key in the list as it stands, moves pop the first
    live element with the value (crdt.py:29-57).  Checked against the list-state
    restatement oracle/rga_list_ref.py on 60 random scripts."""
    from oracle.rga_list_ref import ListRga
    rng = np.random.default_rng(29)
    n_unordered = 0
    for case in range(60):
        r, ref = RGA(), ListRga()
        for st in _out_of_order_script(rng, 30):
            op = st[0]
            if op == "assign":
                r.list = [Elem(Key(*k), v, tb) for k, v, tb in st[1]]
                ref = ListRga([(tuple(k), v, tb) for k, v, tb in st[1]])
            elif op == "append":
                r.list.append(Elem(Key(*st[1]), st[2], st[3]))
                ref.rows.append([tuple(st[1]), st[2], st[3]])
            elif op == "reverse":
                r.list.reverse()
                ref.rows.reverse()
            elif op == "insert":
                r.insert(Key(*st[2]), st[1])
                ref.insert(tuple(st[2]), st[1])
            elif op == "move":
                r.move(st[1], Key(*st[2]))
                ref.move(st[1], tuple(st[2]))
            elif op == "delete":
                r.delete(st[1])
                ref.delete(st[1])
            else:
                got = [((e.key.anchor, e.key.t, e.key.author, e.key.opid), e.value, e.tombstone) for e in r.list]
                assert got == ref.state(), f"script {case}"
                ks = [g[0] for g in got]
                n_unordered += any(b < a for a, b in zip(ks, ks[1:]))
                assert r.materialize() == [v for _, v, tb in got if not tb]
    assert n_unordered > 20  # the scripts do reach states out of key order


@pytest.mark.parametrize("n_ops,n_lists,seed", [(1_000_000, 5_000, 14), (300_000, 30, 15)])
def test_rga_list_mode_live_elements_match(n_ops, n_lists, seed):
    """At scale (the oracle has no list mode): the list state's live elements are exactly
    materialize()'s output, list by list, and its tombstoned ones are extra elements."""
    batch = synth.rga_batch(n_ops, n_lists, seed)
    lv, ls, lo = rga_replay_device(batch)
    tv, ts, to, tomb = rga_replay_device(batch, tombstones=True)
    assert tomb.any()
    for i in range(batch.n_lists):
        a, b = to[i], to[i + 1]
        live = ~tomb[a:b]
        assert np.array_equal(ts[a:b][live], ls[lo[i]:lo[i + 1]]), f"list {i}"
        assert np.array_equal(tv[a:b][live], lv[lo[i]:lo[i + 1]])
    assert np.all(batch.op[ts[tomb]] != 2)  # tombstoned elements were created by inserts / moves


def _check(batch, grouped=False):
    gv, gs, go = rga_replay_device(batch, grouped=grouped)
    ov, os_, oo = oracle.rga(batch.n_lists, batch.list_id, batch.op, batch.value, batch.anchor,
                             batch.t, batch.author, batch.opid_hi, batch.opid_lo)
    assert np.array_equal(go, oo)
    assert np.array_equal(gs, os_)
    assert np.array_equal(gv, ov)


@pytest.mark.parametrize("n_ops,n_lists,seed", [(200_000, 1_000, 13), (1_000_000, 5_000, 14),
                                                (400_000, 100_000, 16),  # > 65536 lists: multi-block scan
                                                (300_000, 65_536, 17),   # the most lists k_rga_out_fused takes
                                                (300_000, 30, 15)])
def test_rga_batch_equals_oracle(n_ops, n_lists, seed):
    _check(synth.rga_batch(n_ops, n_lists, seed))


@pytest.mark.timeout(300)
def test_rga_config4_full_size():
    """SURVEY §8(d) config 4 at its full size: 10M events over 50k lists, seed 13."""
    _check(synth.rga_batch(10_000_000, 50_000, 13))


def _grouped(b):
    """The same lists with each list's events together, in stream order (the shape
    crdt.replay and RGA hand the library): a stable sort by list id, events re-indexed."""
    from semantic_merge_amd.crdt import RgaBatch
    p = np.argsort(b.list_id, kind="stable")
    return RgaBatch(b.n_lists, b.list_id[p], b.op[p], b.value[p], b.anchor[p], b.t[p], b.author[p],
                    b.opid_hi[p], b.opid_lo[p], [])


@pytest.mark.timeout(300)
def test_rga_config4_grouped_full_size():
    """Config 4's 10M events over 50k lists, grouped list by list (the drop-in's shape):
    the SMX_RGA_GROUPED path (records packed in place, no partition) against the C oracle."""
    _check(_grouped(synth.rga_batch(10_000_000, 50_000, 13)), grouped=True)


@pytest.mark.parametrize("n_ops,n_lists,seed", [(300_000, 1_000, 21), (200_000, 100_000, 22), (50_000, 30, 23)])
def test_rga_grouped_equals_oracle(n_ops, n_lists, seed):
    """Grouped batches with empty lists at the start, in the middle and at the end (list
    ids from a sparse subset), and more lists than k_rga_out_fused takes."""
    b = _grouped(synth.rga_batch(n_ops, n_lists, seed))
    keep = (b.list_id % 3 != 0) & (b.list_id != b.n_lists - 1)
    from semantic_merge_amd.crdt import RgaBatch
    b = RgaBatch(b.n_lists, *(x[keep] for x in (b.list_id, b.op, b.value, b.anchor, b.t, b.author, b.opid_hi,
                                                 b.opid_lo)), [])
    assert b.list_id[0] > 0 and b.list_id[-1] < b.n_lists - 1
    _check(b, grouped=True)


def test_rga_grouped_claim_false_still_exact():
    """SMX_RGA_GROUPED on interleaved events: the device check sees a list id decrease,
    the list kernels stand down and the call redoes itself through the partition."""
    _check(synth.rga_batch(400_000, 2_000, 24), grouped=True)


def test_rga_grouped_invalid_input():
    b = _grouped(synth.rga_batch(100_000, 50, 25))
    b.list_id[-1] = 50  # out of range (last: the ids still never decrease)
    with pytest.raises(Exception, match="n_lists"):
        rga_replay_device(b, grouped=True)
    b = _grouped(synth.rga_batch(100_000, 50, 25))
    b.op[777] = 3
    with pytest.raises(Exception, match="op > 2"):
        rga_replay_device(b, grouped=True)


def test_rga_dense_values_and_big_lists():
    # few values per list (long per-value chains) and lists beyond the LDS capacity
    _check(synth.rga_batch(60_000, 8, 16, values_per_list=3, anchors_per_list=2, authors=1))


def test_rga_mixed_list_sizes():
    # empty lists, ~100-event lists (LDS kernel), ~2000-event lists on both sides of the
    # 2048 boundary (large LDS kernel / global path) and one ~20k-event list (global path)
    b = synth.rga_batch(400_000, 2_000, 17)
    lid = b.list_id.astype(np.int64)
    lid = np.where(lid < 400, lid % 40, lid)
    lid = np.where(lid >= 1900, 1999, lid)
    b.list_id = lid.astype(np.uint32)
    counts = np.bincount(lid, minlength=2000)
    assert (counts > 2048).any() and ((counts > 512) & (counts <= 2048)).any() and (counts == 0).any()
    _check(b)


def test_rga_hot_list_and_invalid_input():
    b = synth.rga_batch(300_000, 50, 18)
    b.list_id[100_000:120_000] = 7  # a run of one list: slot atomics aggregate per wave
    _check(b)
    b.list_id[5] = 50
    with pytest.raises(Exception, match="n_lists"):
        rga_replay_device(b)
    b.list_id[5] = 7
    b.op[200_001] = 3  # an op beyond delete (checked by the partition's first pass)
    with pytest.raises(Exception, match="op > 2"):
        rga_replay_device(b)


def test_rga_lists_at_capacity_all_values_distinct():
    """Lists of exactly 256 events (k_rga_wave's capacity) whose values are all distinct:
    the list kernel's value hash table (one slot per event) fills completely; and lists
    of 257 events (the deferred kernel)."""
    b = synth.rga_batch(400 * 256 + 300 * 257, 700, 19)
    rng = np.random.default_rng(19)
    lid = np.concatenate([np.repeat(np.arange(400), 256), np.repeat(np.arange(400, 700), 257)])
    rng.shuffle(lid)
    b.list_id = lid.astype(np.uint32)
    b.value = np.arange(lid.size, dtype=np.uint32)  # distinct everywhere (first-seen order)
    _check(b)


def test_rga_key_ranges_packed_and_wide_sorts():
    """The list kernels sort survivors on 32-bit packed keys when a list's anchor and t
    ranges fit beside the event bits (31 bits in all), on 64-bit keys otherwise: lists on
    both sides of that line, full-range signed t, 32-bit anchors, and equal top halves
    of t (ties on word 0 resolved by the full key)."""
    b = synth.rga_batch(400_000, 2_000, 21)
    rng = np.random.default_rng(21)
    lid = b.list_id.astype(np.int64)
    n = lid.size
    reg = lid % 6
    t = b.t.copy()
    anchor = b.anchor.astype(np.int64)
    full_t = rng.integers(-(1 << 63), (1 << 63) - 1, size=n, dtype=np.int64, endpoint=True)
    t = np.where(reg == 0, full_t, t)
    anchor = np.where(reg == 1, rng.integers(0, 1 << 32, size=n, dtype=np.int64), anchor)
    low = rng.integers(0, 1 << 32, size=n, dtype=np.int64)
    # 11 anchor bits + 12 t bits + 8 event bits = 31 (packed); 11 + 13 + 8 = 32 (64-bit keys)
    for r, tb in ((2, 12), (3, 13)):
        sel = reg == r
        a = np.where(rng.random(n) < 0.5, 0, (1 << 11) - 1)
        hi = rng.integers(0, 1 << tb, size=n, dtype=np.int64)
        hi = np.where(rng.random(n) < 0.1, (1 << tb) - 1, hi)
        anchor = np.where(sel, a + 5, anchor)
        t = np.where(sel, (hi << 32) | low, t)
    # equal top halves of t inside a list: word-0 ties broken by the low half, author, opid
    sel = reg == 4
    t = np.where(sel, (rng.integers(0, 3, size=n, dtype=np.int64) << 32) | low, t)
    anchor = np.where(sel, anchor % 2, anchor)
    b.t = t
    b.anchor = anchor.astype(np.uint32)
    _check(b)
