"""The CPU oracle (oracle/compose_ref.c) reproduces the reference's own outputs.

Golden vectors come from running the reference in the build container
(tools/make_golden.py); this pins the oracle before anything is checked against it.
"""
import hashlib

import pytest

from oracle import oracle
from semantic_merge_amd import synth
from semantic_merge_amd.marshal import marshal
from semantic_merge_amd.materialize import materialize_conflicts, materialize_ops

from _util import assert_case, jline, load, to_ops


def test_scenarios_match_reference():
    for name, case in load("compose_scenarios.json").items():
        assert_case(oracle.compose, case, name)


def test_edge_cases_match_reference():
    cases = load("compose_cases.json")
    assert len(cases) >= 500
    for i, case in enumerate(cases):
        assert_case(oracle.compose, case, f"case {i}")


def _digest(dicts):
    h = hashlib.sha256()
    for d in dicts:
        h.update(jline(d).encode("utf-8"))
        h.update(b"\n")
    return h.hexdigest()


def spec_of(rec):
    kw = dict(rec["spec"])
    kw["mix"] = tuple(tuple(x) for x in rec["mix"])
    return synth.LiftSpec(**kw)


@pytest.mark.parametrize("name", ["lift_20k", "lift_100k_shuffled", "adversarial_100k",
                                  "lift_200k", "c2_1M"])
def test_synthetic_digests_match_reference(name):
    rec = {r["name"]: r for r in load("compose_digests.json")}[name]
    logs = synth.lift_logs(spec_of(rec))
    A, B = synth.lift_op_dicts(logs)
    oa, ob = to_ops(A), to_ops(B)
    soa = marshal(oa, ob)
    order, addr, file, ctx, pairs = oracle.compose(soa)
    allops = oa + ob
    out = materialize_ops(allops, soa.kind, soa.strings, order, addr, file, ctx)
    conf = materialize_conflicts(allops, pairs)
    assert len(out) == rec["n_out"] and len(conf) == rec["n_conflicts"]
    assert _digest(o.to_dict() for o in out) == rec["out_sha256"]
    assert _digest(c.to_dict() for c in conf) == rec["conflicts_sha256"]
