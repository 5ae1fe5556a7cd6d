"""GPU parity: libsmx (through the C ABI) == reference golden vectors == CPU oracle."""
import hashlib

import numpy as np
import pytest

from oracle import oracle
from semantic_merge_amd import synth
from semantic_merge_amd._lib import DeviceCompose, compose_soa
from semantic_merge_amd.compose import compose_oplogs
from semantic_merge_amd.marshal import marshal

from _util import assert_case, jline, load, to_ops

pytestmark = pytest.mark.gpu


def _eq_soa(gpu, ref, label):
    names = ("order", "addr", "file", "ctx", "conflicts")
    for name, g, r in zip(names, gpu, ref):
        assert g.shape == r.shape, f"{label}: {name} shape {g.shape} vs {r.shape}"
        if not np.array_equal(g, r):
            bad = np.flatnonzero(g.reshape(-1) != r.reshape(-1))[:5]
            raise AssertionError(f"{label}: {name} differs at {bad.tolist()}")


def test_library_runs_on_gpu():
    import torch
    assert torch.cuda.is_available()
    soa = synth.lift_soa(synth.lift_logs(synth.LiftSpec(5000, 50, 1)))
    _eq_soa(compose_soa(soa), oracle.compose(soa), "lift_5k")


def test_scenarios_gpu():
    for name, case in load("compose_scenarios.json").items():
        assert_case(compose_soa, case, name)


def test_edge_cases_gpu():
    for i, case in enumerate(load("compose_cases.json")):
        assert_case(compose_soa, case, f"case {i}")


def test_edge_cases_dropin_gpu():
    """All 600 reference cases through the drop-in itself: native marshal straight into the
    session's pinned staging columns (and the Python encoders' replacement columns when
    timestamps or ids are not ISO / canonical), the device merge, native materialise from
    the staging area's views, the conflicts -- on Op objects, as the CLI calls it."""
    for i, case in enumerate(load("compose_cases.json")):
        A, B = to_ops(case["A"]), to_ops(case["B"])
        out, conf = compose_oplogs(A, B)
        assert jline([o.to_dict() for o in out]) == jline(case["out"]), f"case {i}: composed ops differ"
        assert jline([c.to_dict() for c in conf]) == jline(case["conflicts"]), f"case {i}: conflicts differ"


def test_dropin_compose_oplogs_matches_reference():
    case = load("compose_scenarios.json")["e2e_rename_move_decl"]
    A, B = to_ops(case["A"]), to_ops(case["B"])
    before = jline([o.to_dict() for o in A + B])
    out, conf = compose_oplogs(A, B)
    assert jline([o.to_dict() for o in out]) == jline(case["out"])
    assert conf == []
    assert jline([o.to_dict() for o in A + B]) == before  # inputs untouched
    ren = [o for o in out if o.type == "renameSymbol"][0]
    assert ren.params["file"] == "lib/util.ts" and ren.params["newFile"] == "lib/util.ts"
    assert all(o is not a for o in out for a in A + B)


def test_config1_e2e_compose_then_apply(tmp_path):
    """Config 1 (/root/reference/tests/e2e_rename_move_decl.sh:14-74) on the box: the GPU
    drop-in compose_oplogs, then the fast apply_ops (semantic_merge_amd/applier.py), give
    the composed log and the merged tree the reference's compose_oplogs + apply_ops gave
    (tests/golden/e2e_tree.json, tools/make_golden.py --only e2e)."""
    import os
    import shutil
    from semantic_merge_amd import applier
    case = load("e2e_tree.json")
    base = tmp_path / "base"
    for pth, text in case["base"].items():
        (base / pth).parent.mkdir(parents=True, exist_ok=True)
        (base / pth).write_text(text, encoding="utf-8")
    out, conf = compose_oplogs(to_ops(case["A"]), to_ops(case["B"]))
    assert jline([o.to_dict() for o in out]) == jline(case["out"])
    assert [c.to_dict() for c in conf] == case["conflicts"] == []
    merged = applier.apply_ops(base, out)
    try:
        files, dirs = {}, []
        for dp, _, fn in os.walk(merged):
            rel = os.path.relpath(dp, merged)
            if rel != ".":
                dirs.append(rel)
            for f in fn:
                with open(os.path.join(dp, f), "rb") as fh:
                    files[os.path.normpath(os.path.join(rel, f))] = fh.read().decode("latin-1")
        assert files == case["files"] and sorted(dirs) == case["dirs"]
        assert "function bar" in files["lib/util.ts"]
    finally:
        shutil.rmtree(merged)


def _digest(dicts):
    h = hashlib.sha256()
    for d in dicts:
        h.update(jline(d).encode("utf-8"))
        h.update(b"\n")
    return h.hexdigest()


@pytest.mark.parametrize("name", ["lift_20k", "lift_100k_shuffled", "adversarial_100k",
                                  "lift_200k", "c2_1M"])
def test_synthetic_digests_gpu(name):
    rec = {r["name"]: r for r in load("compose_digests.json")}[name]
    kw = dict(rec["spec"])
    kw["mix"] = tuple(tuple(x) for x in rec["mix"])
    logs = synth.lift_logs(synth.LiftSpec(**kw))
    A, B = synth.lift_op_dicts(logs)
    out, conf = compose_oplogs(to_ops(A), to_ops(B))
    assert len(out) == rec["n_out"] and len(conf) == rec["n_conflicts"]
    assert _digest(o.to_dict() for o in out) == rec["out_sha256"]
    assert _digest(c.to_dict() for c in conf) == rec["conflicts_sha256"]


@pytest.mark.parametrize("spec", [
    synth.LiftSpec(1_000_000, 10_000, 7),                       # config 2
    synth.LiftSpec(1_000_000, 10_000, 7, shuffle=True),         # robustness variant
    synth.LiftSpec(2_000_000, 2_000, 17, ops_per_ms=4096, mix=synth.ADVERSARIAL_MIX,
                   rename_overlap=0.30),                         # config 5 shape
    synth.LiftSpec(1_000_000, 64, 23, ops_per_ms=16, mix=synth.ADVERSARIAL_MIX),  # hot symbols
    synth.LiftSpec(333_333, 1, 29, ops_per_ms=1),               # one symbol, every head collides
    synth.LiftSpec(1_000_000, 1_000, 41, ops_per_ms=160),       # windows overflow -> smaller windows
    synth.LiftSpec(400_000, 5_000_000, 43),                     # > 4M symbols: atomic tables
    synth.LiftSpec(600_000, 2_000, 61, ops_per_ms=3000, mix=synth.ADVERSARIAL_MIX),  # wide windows
    synth.LiftSpec(300_000, 500, 59, ops_per_ms=10_000),        # groups too long: radix plan
], ids=["c2_1M", "c2_1M_shuffled", "c5_2M", "hot64_1M", "onesym", "dense160", "sym5M", "wide3000",
        "groups10k"])
def test_gpu_equals_oracle_soa(spec):
    soa = synth.lift_soa(synth.lift_logs(spec))
    _eq_soa(compose_soa(soa), oracle.compose(soa), str(spec))


@pytest.mark.parametrize("stretch", ["all", "half"])
def test_gpu_wide_timestamp_range(stretch):
    """Timestamps far apart (windows spanning more than 2^32 key units: every window
    ("all") or the windows across a 2^40 jump ("half")): the presorted plan's u64
    window keys order them exactly."""
    soa = synth.lift_soa(synth.lift_logs(synth.LiftSpec(400_000, 2_000, 71)))
    for lo, m in ((0, soa.n_a), (soa.n_a, soa.n_b)):
        ts = soa.ts[lo:lo + m].copy()
        rank = np.searchsorted(np.unique(ts), ts).astype(np.uint64)
        if stretch == "all":
            soa.ts[lo:lo + m] = rank * np.uint64(1 << 33) + np.uint64(5)
        else:  # a jump of 2^40 halfway: the windows that straddle it span it
            soa.ts[lo:lo + m] = rank + np.where(np.arange(m) >= m // 2, np.uint64(1 << 40), np.uint64(0))
    assert np.all(np.diff(soa.ts[:soa.n_a].astype(np.float64)) >= 0)
    dc = DeviceCompose(soa)
    dc.run()
    _eq_soa(dc.results(), oracle.compose(soa), f"wide timestamps ({stretch})")
    assert dc.last_plan() == "presorted"


def test_gpu_wide_plan_config5_shape():
    """Config-5-shaped log (ordered, 8192-op timestamp groups over both branches): no
    2048-op window holds a group, the wide (8192-op) presorted windows do."""
    soa = synth.lift_soa(synth.lift_logs(synth.LiftSpec(1_000_000, 3_000, 17, ops_per_ms=4096,
                                                         mix=synth.ADVERSARIAL_MIX, rename_overlap=0.30)))
    dc = DeviceCompose(soa)
    dc.run()
    _eq_soa(dc.results(), oracle.compose(soa), "config 5 shape, wide windows")
    assert dc.last_plan() == "presorted-wide"


def _alternating_groups(spec, big, small):
    """spec's logs with timestamp groups of alternately `big` and `small` ops per branch
    (the same on both branches)."""
    soa = synth.lift_soa(synth.lift_logs(spec))
    for lo, m in ((0, soa.n_a), (soa.n_a, soa.n_b)):
        period = big + small
        k = np.arange(m)
        grp = 2 * (k // period) + ((k % period) >= big)
        soa.ts[lo:lo + m] = soa.ts[0] + grp.astype(np.uint64) * np.uint64(2)
    return soa


def test_gpu_segmented_plan_when_wide_windows_overflow():
    """Groups of 8100 and 200 ops (4050 + 4050, 100 + 100) in turn: a window that holds
    a large group and the small one after it overflows even the wide window at every
    target size, so the segmented sort (each branch's groups <= 4096) orders the log."""
    soa = _alternating_groups(synth.LiftSpec(500_000, 2_000, 73, mix=synth.ADVERSARIAL_MIX), 4050, 100)
    dc = DeviceCompose(soa)
    dc.run()
    _eq_soa(dc.results(), oracle.compose(soa), "alternating 8100 / 200 groups")
    assert dc.last_plan() == "segmented"


@pytest.mark.parametrize("shape,plan", [("c5", "presorted-wide"), ("alt8100", "segmented"), ("long20000", "radix")])
def test_gpu_early_verdict_plans(shape, plan):
    """Merges from 4M ops take the synchronous early verdict: k_khist tests the groups,
    k_fpart places the wide plan's boundaries on F_LONG and the host launches the wide
    windows; when even those overflow (groups of 8100 + 200 in turn), or k_fpart's wide
    test fails (20000-op groups: F_WLONG), the fallbacks take over from the meta."""
    spec = synth.LiftSpec(4_500_000, 20_000, 79, mix=synth.ADVERSARIAL_MIX)
    if shape == "c5":
        soa = synth.lift_soa(synth.lift_logs(synth.LiftSpec(4_500_000, 20_000, 79, ops_per_ms=4096,
                                                             mix=synth.ADVERSARIAL_MIX)))
    elif shape == "alt8100":
        soa = _alternating_groups(spec, 4050, 100)
    else:
        soa = _alternating_groups(spec, 10000, 10000)
    assert soa.n >= (1 << 22)
    dc = DeviceCompose(soa)
    dc.run()
    _eq_soa(dc.results(), oracle.compose(soa), f"early verdict, {shape}")
    assert dc.last_plan() == plan


def test_gpu_segmented_plan_duplicate_ids():
    """Config-5-shaped log (ordered, 4096-op timestamp groups per branch: the wide
    windows) with duplicate ids and ids equal in their top bits inside groups: equal
    32-bit rank keys are ranked on the full id, then by index, in the rank loop; and the
    same ids under the segmented sort (groups of 4050 and 100 ops per branch in turn),
    whose tie runs are re-sorted on the full id, then by index."""
    for label, soa in (
            ("wide", synth.lift_soa(synth.lift_logs(synth.LiftSpec(400_000, 1_000, 67, ops_per_ms=4096,
                                                                    mix=synth.ADVERSARIAL_MIX)))),
            ("segmented", _alternating_groups(synth.LiftSpec(400_000, 1_000, 67, mix=synth.ADVERSARIAL_MIX),
                                              4050, 100))):
        _dup_ids(soa)
        dc = DeviceCompose(soa)
        dc.run()
        _eq_soa(dc.results(), oracle.compose(soa), f"{label} plan, duplicate ids")
        assert dc.last_plan() == ("presorted-wide" if label == "wide" else "segmented")


def _dup_ids(soa):
    rng = np.random.default_rng(67)
    n = soa.n
    dup = rng.choice(n - 1, 3000, replace=False)
    soa.oid_hi[dup + 1] = soa.oid_hi[dup]            # same top bits (and same hi) as a neighbour
    both = dup[:1000]
    soa.oid_lo[both + 1] = soa.oid_lo[both]          # duplicate ids
    near = rng.choice(n, 2000, replace=False)
    soa.oid_hi[near] = (soa.oid_hi[near] & ~np.uint64(0x1fff)) | np.uint64(7)  # equal above bit 13


@pytest.mark.parametrize("plan", ["presorted-wide", "segmented"])
def test_gpu_long_groups_clustered_ids(plan):
    """Ids whose top bits cluster (sequential ids in the first half of each branch, as
    short string ids give; distinct in the 38 sorted bits, so no tie runs), in long
    timestamp groups: the wide windows' interpolation buckets crowd; the segmented
    sort's tiles overflow their buckets and take the bitonic network, the random-id
    tiles keep the buckets."""
    spec = synth.LiftSpec(400_000, 1_000, 71, ops_per_ms=4096, mix=synth.ADVERSARIAL_MIX)
    soa = (synth.lift_soa(synth.lift_logs(spec)) if plan == "presorted-wide"
           else _alternating_groups(spec, 4050, 100))
    for lo, hi in ((0, soa.n_a // 2), (soa.n_a, soa.n_a + soa.n_b // 2)):
        seq = np.arange(hi - lo, dtype=np.uint64)
        soa.oid_hi[lo:hi] = ((seq * np.uint64(2654435761)) & np.uint64(0xFFFFF)) << np.uint64(26)
    _eq_soa(compose_soa(soa), oracle.compose(soa), f"{plan} plan, clustered ids")
    assert DeviceCompose.last_plan() == plan


def test_gpu_segmented_sort_fails_then_radix():
    """Ordered logs whose timestamp groups (10k ops) exceed the segmented sort's tiles:
    the sort flags the plan failed, the kernels queued behind it (windows, walk, tables,
    emit) leave at once, and the merge's meta read sends it to the radix plan."""
    soa = synth.lift_soa(synth.lift_logs(synth.LiftSpec(300_000, 500, 59, ops_per_ms=10_000)))
    dc = DeviceCompose(soa)
    dc.run()
    _eq_soa(dc.results(), oracle.compose(soa), "segmented sort fails, radix plan")
    assert dc.last_plan().startswith("radix")


@pytest.mark.parametrize("bits", [15, 20, 31], ids=["packed48", "packed64", "wide"])
def test_gpu_value_widths(bits):
    """Value ids of `bits` bits: 3 x 15 fits the 6-byte final-state table entries,
    3 x 20 the 8-byte ones, 3 x 31 neither (int4 table)."""
    soa = synth.lift_soa(synth.lift_logs(synth.LiftSpec(300_000, 3_000, 47)))
    rng = np.random.default_rng(bits)
    hi = np.int64(1) << (bits - 1)
    for v in (soa.v0, soa.v1):
        m = v >= 0
        v[m] = (hi + rng.integers(0, hi, m.sum())).astype(np.int32)
    _eq_soa(compose_soa(soa), oracle.compose(soa), f"value bits {bits}")


def test_gpu_repeatable_and_none_moves():
    spec = synth.LiftSpec(300_000, 3_000, 31)
    soa = synth.lift_soa(synth.lift_logs(spec))
    rng = np.random.default_rng(5)
    mv = np.flatnonzero(soa.kind == 0)
    soa.v0[rng.choice(mv, len(mv) // 3, replace=False)] = -1   # None newAddress
    soa.v1[rng.choice(mv, len(mv) // 4, replace=False)] = -1   # falsy newFile and file
    dc = DeviceCompose(soa)
    dc.run()
    first = dc.results()
    dc.run()
    second = dc.results()
    ref = oracle.compose(soa)
    _eq_soa(first, ref, "none-moves")
    _eq_soa(second, ref, "none-moves rerun")


def test_invalid_input_fails_loudly():
    from semantic_merge_amd._lib import SmxError
    soa = synth.lift_soa(synth.lift_logs(synth.LiftSpec(10_000, 100, 2)))
    soa.sym[7] = soa.n_sym + 3
    with pytest.raises(SmxError):
        compose_soa(soa)
    soa = synth.lift_soa(synth.lift_logs(synth.LiftSpec(10_000, 100, 2)))
    soa.kind[11] = 40
    with pytest.raises(SmxError):
        compose_soa(soa)


def _chain(n_ren, seed, interleave):
    """One DivergentRename region as long as the logs: every op renames symbol 0.  A's
    renames all take name class 0; B's class 1 (every head pair conflicts) or, with
    interleave, a random class per rename and interleaved timestamps (equal names do
    not conflict, so the pairing drifts along the chain)."""
    from semantic_merge_amd.marshal import SoA
    rng = np.random.default_rng(seed)
    na = nb = n_ren
    kind = np.full(na + nb, 1, np.uint8)
    if interleave:
        ts = np.concatenate([np.arange(na, dtype=np.uint64) * 2, np.arange(nb, dtype=np.uint64) * 2 + 1])
    else:
        ts = np.concatenate([np.arange(na, dtype=np.uint64), np.uint64(na) + np.arange(nb, dtype=np.uint64)])
    hi = rng.integers(0, 2**63, size=na + nb, dtype=np.int64).astype(np.uint64)
    lo = rng.integers(0, 2**63, size=na + nb, dtype=np.int64).astype(np.uint64)
    sym = np.zeros(na + nb, np.uint32)
    v0 = np.concatenate([np.zeros(na, np.int32),
                         rng.integers(0, 2, nb).astype(np.int32) if interleave else np.ones(nb, np.int32)])
    v1 = v0.copy()
    return SoA(na, nb, kind, ts, hi, lo, sym, v0, v1, 1, ["a", "b"])


@pytest.mark.parametrize("interleave", [False, True])
def test_long_same_symbol_chain_is_linear(interleave):
    """a region of 200k conflicting renames of one symbol goes through the
    capped replay + cluster path; the result equals the oracle and one merge stays
    well under a second (a quadratic replay would take minutes)."""
    import time
    import torch
    soa = _chain(100_000, 3, interleave)
    ref = oracle.compose(soa)
    assert len(ref[4]) > 30_000
    compose_soa(soa)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    got = compose_soa(soa)
    dt = time.perf_counter() - t0
    _eq_soa(got, ref, f"chain interleave={interleave}")
    assert dt < 1.0, f"{dt:.3f} s for 200k chained renames"


def test_compose_json_matches_dropin():
    """oplog.compose_json (JSON texts -> one-pass decode + SoA -> GPU -> Op objects)
    equals compose_oplogs on OpLog.from_json's ops, on the reference's own cases."""
    import json
    from semantic_merge_amd.oplog import OpLog, compose_json
    for i, case in enumerate(load("compose_cases.json")[:120]):
        ta, tb = json.dumps(case["A"]), json.dumps(case["B"])
        out, conf = compose_json(ta, tb)
        assert [o.to_dict() for o in out] == case["out"], f"case {i}"
        assert [c.to_dict() for c in conf] == case["conflicts"], f"case {i}"
        ref = compose_oplogs(OpLog.from_json(ta).ops, OpLog.from_json(tb).ops)
        assert [o.to_dict() for o in ref[0]] == case["out"]


@pytest.mark.parametrize("frac,dup", [(0.3, False), (1.0, True)])
def test_gpu_presorted_id_prefix_ties(frac, dup):
    """Ops whose ids share their top 32 bits (and, with dup, whole ids) inside equal-
    (kind, timestamp) groups: the presorted window's 32-bit group rank collides and the
    window re-ranks exactly on the full ids -- with the renames' ranks computed around
    it (a window with ties and renames)."""
    soa = synth.lift_soa(synth.lift_logs(synth.LiftSpec(300_000, 3_000, 21)))
    rng = np.random.default_rng(5)
    sel = rng.random(soa.n) < frac
    soa.oid_hi[sel] = (soa.oid_hi[sel] & np.uint64(0xFFFFFFFF)) | np.uint64(0x4242424200000000)
    if dup:
        soa.oid_lo[sel] = np.uint64(7)
        soa.oid_hi[sel] &= np.uint64(0xFFFFFFFFFFFF000F)  # many exact duplicates
    dc = DeviceCompose(soa)
    dc.run()
    got = dc.results()
    assert DeviceCompose.last_plan() == "presorted"
    _eq_soa(got, oracle.compose(soa), f"id prefix ties frac={frac} dup={dup}")


def test_dropin_reentrant_merge_from_materialise():
    """A merge started while the drop-in materialises (here from a value's __deepcopy__,
    which the native copier hands to copy.deepcopy) gets buffers of its own: the outer
    merge's results, read as views of the thread's staging area, stay intact."""
    import copy
    case = load("compose_scenarios.json")["e2e_rename_move_decl"]
    inner = [to_ops(c["A"]) for c in load("compose_cases.json")[:2]]

    class Hook:
        calls = 0

        def __init__(self, tag, nested):
            self.tag, self.nested = tag, nested

        def __deepcopy__(self, memo):
            if self.nested:
                compose_oplogs(inner[0], inner[1])
                Hook.calls += 1
            return Hook(self.tag, self.nested)

        def __eq__(self, other):
            return isinstance(other, Hook) and other.tag == self.tag

    def run(nested):
        A, B = to_ops(case["A"]), to_ops(case["B"])
        for i, o in enumerate(A + B):
            o.guards = {**o.guards, "hook": Hook(i, nested)}
        out, conf = compose_oplogs(A, B)
        return [(o.id, o.type, o.target.addressId, dict(o.params), o.guards["hook"].tag) for o in out], conf

    Hook.calls = 0
    want = run(False)
    got = run(True)
    assert Hook.calls > 0
    assert got == want
    assert [(i, t, a, p) for i, t, a, p, _ in want[0]] == [
        (d["id"], d["type"], d["target"]["addressId"], d["params"]) for d in case["out"]]
