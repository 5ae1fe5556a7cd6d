"""GPU parity of the small-merge plan (SMX_PLAN_SMALL, smx_small.h: merges of at most 2048
ops in one workgroup) against the golden vectors and the CPU oracle, and the same cases
forced through the window plans (smx_set_small_limit(0)) so both paths stay covered."""
import numpy as np
import pytest

from oracle import oracle
from semantic_merge_amd import synth
from semantic_merge_amd._lib import DeviceCompose, compose_soa, set_small_limit

from _util import assert_case, load

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["small", "windows"])
def plan(request):
    old = set_small_limit(2048 if request.param == "small" else 0)
    yield request.param
    set_small_limit(old)


def _eq(gpu, ref, label):
    for name, g, r in zip(("order", "addr", "file", "ctx", "conflicts"), gpu, ref):
        assert g.shape == r.shape, f"{label}: {name} shape {g.shape} vs {r.shape}"
        if not np.array_equal(g, r):
            bad = np.flatnonzero(g.reshape(-1) != r.reshape(-1))[:5]
            raise AssertionError(f"{label}: {name} differs at {bad.tolist()}")


def test_golden_both_plans(plan):
    for name, case in load("compose_scenarios.json").items():
        assert_case(compose_soa, case, f"{plan} {name}")
    for i, case in enumerate(load("compose_cases.json")):
        assert_case(compose_soa, case, f"{plan} case {i}")


SPECS = [
    synth.LiftSpec(1, 1, 3),
    synth.LiftSpec(2, 1, 4),
    synth.LiftSpec(17, 3, 5, ops_per_ms=1),
    synth.LiftSpec(1000, 100, 6),
    synth.LiftSpec(1000, 20, 7, shuffle=True),
    synth.LiftSpec(2000, 30, 8, ops_per_ms=4096, mix=synth.ADVERSARIAL_MIX, rename_overlap=1.0),
    synth.LiftSpec(2047, 5, 9, ops_per_ms=1, mix=synth.ADVERSARIAL_MIX, divergent=0.5),
    synth.LiftSpec(2048, 2048, 10, shuffle=True, mix=synth.ADVERSARIAL_MIX),
    synth.LiftSpec(2048, 1, 12, ops_per_ms=1),
]


@pytest.mark.parametrize("spec", SPECS, ids=lambda s: f"{s.n_total}x{s.n_sym}s{s.seed}")
def test_synthetic_small(plan, spec):
    soa = synth.lift_soa(synth.lift_logs(spec))
    _eq(compose_soa(soa), oracle.compose(soa), f"{plan} {spec}")
    assert (DeviceCompose.last_plan() == "small") == (plan == "small")


def test_size_boundary():
    """2048 ops take the small plan, 2049 the window plans; both match the oracle."""
    for n, small in ((2048, True), (2049, False)):
        soa = synth.lift_soa(synth.lift_logs(synth.LiftSpec(n, 40, 13, mix=synth.ADVERSARIAL_MIX)))
        _eq(compose_soa(soa), oracle.compose(soa), f"n={n}")
        assert (DeviceCompose.last_plan() == "small") == small


def test_invalid_symbol_fails(plan):
    soa = synth.lift_soa(synth.lift_logs(synth.LiftSpec(300, 10, 14)))
    soa.sym[5] = soa.n_sym  # out of range
    with pytest.raises(Exception):
        compose_soa(soa)


def test_verdict_word_sequence():
    """Synchronous calls read the merge's verdict word (the last kernel's seq << 1 | bit in
    pinned host memory) instead of the meta block: failures and successes of both plans,
    interleaved on one thread, each see their own verdict."""
    def soa_of(n, seed, bad=False):
        soa = synth.lift_soa(synth.lift_logs(synth.LiftSpec(n, max(n // 20, 1), seed, mix=synth.ADVERSARIAL_MIX)))
        if bad:
            soa.sym[n // 2] = soa.n_sym
        return soa

    seq = [(300, False), (300, True), (1000, False), (5000, False), (5000, True), (700, False),
           (5000, False), (2048, True), (2048, False)]
    for i, (n, bad) in enumerate(seq):
        soa = soa_of(n, 40 + i, bad)
        if bad:
            with pytest.raises(Exception):
                compose_soa(soa)
        else:
            _eq(compose_soa(soa), oracle.compose(soa), f"step {i}: n={n}")
            assert (DeviceCompose.last_plan() == "small") == (n <= 2048)


@pytest.mark.parametrize("shape", ["file_none", "addr_none", "mixed", "one_symbol"])
def test_none_valued_moves(plan, shape):
    """Moves whose newAddress or newFile is None see their symbol's inclusive prefix of
    non-None values (compose.py:73-82): whole histories without a file, without an address,
    None values mixed in, and one symbol whose ~500 moves chain through every step of the
    small plan's prefix pass (was a backwards scan per move)."""
    spec = synth.LiftSpec(2048, 1 if shape == "one_symbol" else 64, 21, ops_per_ms=3)
    soa = synth.lift_soa(synth.lift_logs(spec))
    rng = np.random.default_rng(5)
    mv = np.flatnonzero(soa.kind == synth.KIND_RANK["moveDecl"])
    if shape == "file_none":
        soa.v1[mv[soa.sym[mv] % 2 == 0]] = -1  # half the symbols never have a file
    elif shape == "addr_none":
        soa.v0[mv[soa.sym[mv] % 3 == 0]] = -1
    else:
        soa.v0[mv[rng.random(len(mv)) < 0.6]] = -1
        soa.v1[mv[rng.random(len(mv)) < 0.6]] = -1
    _eq(compose_soa(soa), oracle.compose(soa), f"{plan} {shape}")
