"""Shared helpers: golden fixtures -> ops -> (marshal, compose backend, materialize) -> JSON."""
import json
import os

import numpy as np

from semantic_merge_amd.marshal import marshal
from semantic_merge_amd.materialize import materialize_conflicts, materialize_ops
from semantic_merge_amd.ops import Op

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLD, name)) as fh:
        return json.load(fh)


def to_ops(dicts):
    return [Op.from_dict(d) for d in dicts]


def jline(obj):
    return json.dumps(obj, ensure_ascii=False, separators=(",", ":"))


def run_backend(backend, A, B):
    """backend(soa) -> (order, addr, file, ctx, pairs); returns (out_dicts, conflict_dicts)."""
    oa, ob = to_ops(A), to_ops(B)
    soa = marshal(oa, ob)
    order, addr, file, ctx, pairs = backend(soa)
    allops = oa + ob
    out = materialize_ops(allops, soa.kind, soa.strings, order, addr, file, ctx)
    conf = materialize_conflicts(allops, np.asarray(pairs).reshape(-1, 2))
    return [o.to_dict() for o in out], [c.to_dict() for c in conf]


def assert_case(backend, case, label=""):
    out, conf = run_backend(backend, case["A"], case["B"])
    assert jline(out) == jline(case["out"]), f"{label}: composed ops differ"
    assert jline(conf) == jline(case["conflicts"]), f"{label}: conflicts differ"
