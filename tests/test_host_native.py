"""The native host marshal / materialise (csrc/smx_host.cpp) against the reference's
golden outputs and against the Python restatement (marshal.py / materialize.py) on the
value-semantics corners: NaN / container newNames, non-ISO timestamps, non-UUID ids,
mapping subclasses, shared containers under deepcopy, custom Op classes.  CPU only."""
import copy
import dataclasses
import json
import math
from collections import OrderedDict

import numpy as np
import pytest

from oracle import oracle
from semantic_merge_amd import synth
from semantic_merge_amd.marshal import marshal, marshal_native
from semantic_merge_amd.materialize import (materialize_conflicts, materialize_ops,
                                            materialize_ops_native, smx_host_ctor_mode)
from semantic_merge_amd.ops import Op, Target

from _util import jline, load, to_ops
from test_oracle_golden import _digest, spec_of


def _soa_equal(a, b):
    for f in dataclasses.fields(a):
        x, y = getattr(a, f.name), getattr(b, f.name)
        if isinstance(x, np.ndarray):
            assert x.dtype == y.dtype and np.array_equal(x, y), f.name
        else:
            assert x == y, f.name


def _native(oa, ob):
    soa = marshal_native(oa, ob)
    _soa_equal(soa, marshal(oa, ob))
    order, addr, file, ctx, pairs = oracle.compose(soa)
    ops = oa + ob
    out = materialize_ops_native(ops, soa.kind, soa.strings, order, addr, file, ctx)
    ref = materialize_ops(ops, soa.kind, soa.strings, order, addr, file, ctx)
    assert len(out) == len(ref)
    for o, r in zip(out, ref):
        assert type(o) is type(r) and type(o.target) is type(r.target)
        assert jline(o.to_dict()) == jline(r.to_dict())
    return out, materialize_conflicts(ops, pairs)


def test_golden_cases_native():
    cases = list(load("compose_scenarios.json").values()) + load("compose_cases.json")
    for i, case in enumerate(cases):
        out, conf = _native(to_ops(case["A"]), to_ops(case["B"]))
        assert jline([o.to_dict() for o in out]) == jline(case["out"]), f"case {i}"
        assert jline([c.to_dict() for c in conf]) == jline(case["conflicts"]), f"case {i}"


@pytest.mark.parametrize("name", ["lift_20k", "adversarial_100k"])
def test_synthetic_digests_native(name):
    rec = {r["name"]: r for r in load("compose_digests.json")}[name]
    A, B = synth.lift_op_dicts(synth.lift_logs(spec_of(rec)))
    out, conf = _native(to_ops(A), to_ops(B))
    assert _digest(o.to_dict() for o in out) == rec["out_sha256"]
    assert _digest(c.to_dict() for c in conf) == rec["conflicts_sha256"]


def _op(typ, sym, ts=None, oid=None, **params):
    prov = {"rev": "x"} if ts is None else {"rev": "x", "timestamp": ts}
    return Op(oid if oid is not None else f"id-{sym}-{typ}-{ts}", 1, typ, Target(sym, f"f::{sym}"),
              params, {"g": [1, {"k": None}]}, {}, prov)


def test_newname_value_semantics():
    nan = float("nan")
    A = [_op("renameSymbol", "s1", "2024-01-01T00:00:01Z", newName=nan),
         _op("renameSymbol", "s2", "2024-01-01T00:00:02Z", newName=["a", 1]),
         _op("renameSymbol", "s3", "2024-01-01T00:00:03Z", newName={"x": (1, 2)}),
         _op("renameSymbol", "s4", "2024-01-01T00:00:04Z", newName=1),
         _op("renameSymbol", "s5", "2024-01-01T00:00:05Z"),
         _op("editStmtBlock", "s1", "2024-01-01T00:00:06Z")]
    B = [_op("renameSymbol", "s1", "2024-01-01T00:00:01.500Z", newName=nan),
         _op("renameSymbol", "s2", "2024-01-01T00:00:02.500Z", newName=["a", 1]),
         _op("renameSymbol", "s3", "2024-01-01T00:00:03.500Z", newName={"x": (1, 2)}),
         _op("renameSymbol", "s4", "2024-01-01T00:00:04.500Z", newName=True),
         _op("renameSymbol", "s5", "2024-01-01T00:00:05.500Z", newName=None)]
    _native(A, B)


def test_uncomparable_newname_raises_the_same_error():
    class Opaque:
        __hash__ = None

    A = [_op("renameSymbol", "s1", newName=Opaque())]
    with pytest.raises(TypeError, match="not comparable") as e1:
        marshal(A, [])
    with pytest.raises(TypeError, match="not comparable") as e2:
        marshal_native(A, [])
    assert str(e1.value) == str(e2.value)


@pytest.mark.parametrize("ids", ["uuid", "short", "long", "mixed", "surrogate"])
@pytest.mark.parametrize("ts", ["iso", "other", "missing"])
def test_key_encodings(ids, ts):
    rng = np.random.default_rng(7)
    ops = []
    for k in range(300):
        if ids == "uuid":
            oid = synth._uuid(int(rng.integers(0, 2**63)), int(rng.integers(0, 2**63)))
        elif ids == "short":
            oid = f"op{int(rng.integers(0, 10**6))}é"
        elif ids == "long":
            oid = f"operation-number-{int(rng.integers(0, 10**9))}"
        elif ids == "mixed":
            oid = f"o{k}" if k % 3 else int(rng.integers(0, 1000))
        else:
            oid = f"s{k}\ud800"
        if ts == "iso":
            t = f"2024-01-01T00:00:{int(rng.integers(0, 60)):02d}" + (".123Z" if k % 2 else "Z")
        elif ts == "other":
            t = ["2024-01-01 00:00:00", 17, "2024-01-01T00:00:00Z", "z"][k % 4]
        else:
            t = None
        typ = ["renameSymbol", "moveDecl", "editStmtBlock", "mystery"][k % 4]
        ops.append(_op(typ, f"s{k % 17}", t, oid, newName=f"n{k % 5}", newAddress=f"a{k % 7}",
                       newFile="" if k % 5 == 0 else f"f{k % 3}", file=f"g{k % 4}"))
    if ids == "mixed":  # ints and strs do not order together: both raise the same TypeError
        with pytest.raises(TypeError):
            marshal(ops[:150], ops[150:])
        with pytest.raises(TypeError):
            marshal_native(ops[:150], ops[150:])
        return
    _native(ops[:150], ops[150:])


def test_mapping_subclasses_and_shared_containers():
    class Params(dict):
        def get(self, key, default=None):  # a mapping whose .get the composer must honour
            return "X" + str(super().get(key, default)) if key == "newAddress" else super().get(key, default)

    shared = ["s", {"deep": [1, 2]}]
    p1 = Params(newAddress="a1", newFile="f1")
    A = [Op("i1", 1, "moveDecl", Target("s1"), p1, {"a": shared, "b": shared}, {}, OrderedDict(timestamp="t1")),
         Op("i2", 1, "editStmtBlock", Target("s1"), {"t": (1, [2])}, {}, {"c": {"x": 1.5}}, {"timestamp": "t2"})]
    B = [Op("i3", 1, "renameSymbol", Target("s1"), {"newName": "n"}, {}, {}, {"timestamp": "t0"}),
         Op("i4", 1, "editStmtBlock", Target("s1"), {"cyc": None}, {}, {}, {"timestamp": "t3"})]
    B[1].params["cyc"] = B[1].params  # self-referencing params: deepcopy keeps the cycle
    soa = marshal_native(A, B)
    _soa_equal(soa, marshal(A, B))
    order, addr, file, ctx, _ = oracle.compose(soa)
    ops = A + B
    out = materialize_ops_native(ops, soa.kind, soa.strings, order, addr, file, ctx)
    ref = materialize_ops(ops, soa.kind, soa.strings, order, addr, file, ctx)
    for o, r in zip(out, ref):
        assert type(o.params) is type(r.params) and type(o.provenance) is type(r.provenance)
        assert repr(o) == repr(r)
    mv = next(o for o in out if o.id == "i1")
    assert mv.guards["a"] is mv.guards["b"] and mv.guards["a"] is not shared  # aliasing kept
    cyc = next(o for o in out if o.id == "i4")
    assert cyc.params["cyc"] is not B[1].params and cyc.params is not B[1].params


def test_inputs_untouched_and_outputs_fresh():
    A = [_op("moveDecl", "s1", "2024-01-01T00:00:01Z", newAddress="a", newFile="f"),
         _op("editStmtBlock", "s1", "2024-01-01T00:00:02Z", file="x")]
    B = [_op("renameSymbol", "s1", "2024-01-01T00:00:00Z", newName="n", file="y")]
    before = copy.deepcopy(A + B)
    out, _ = _native(A, B)
    assert A + B == before
    for o in out:
        src = next(x for x in A + B if x.id == o.id)
        assert o is not src and o.params is not src.params and o.guards is not src.guards
        assert o.guards["g"] is not src.guards["g"] and o.guards["g"][1] is not src.guards["g"][1]


@dataclasses.dataclass
class PostOp:
    id: str
    schemaVersion: int
    type: str
    target: Target
    params: dict
    guards: dict
    effects: dict
    provenance: dict
    calls = 0

    def __post_init__(self):
        PostOp.calls += 1

    def to_dict(self):
        return Op.to_dict(self)


@dataclasses.dataclass(frozen=True)
class FrozenTarget:
    symbolId: str
    addressId: str = None

    def to_dict(self):
        return {"symbolId": self.symbolId, "addressId": self.addressId}


class PlainOp:  # not a dataclass: the constructor must be called
    def __init__(self, id, schemaVersion, type, target, params, guards, effects, provenance):
        self.id, self.schemaVersion, self.type, self.target = id, schemaVersion, type, target
        self.params, self.guards, self.effects, self.provenance = params, guards, effects, provenance

    def to_dict(self):
        return Op.to_dict(self)


def test_constructor_modes():
    names = ("id", "schemaVersion", "type", "target", "params", "guards", "effects", "provenance")
    assert smx_host_ctor_mode(Op, names) == 1
    assert smx_host_ctor_mode(Target, ("symbolId", "addressId")) == 1
    assert smx_host_ctor_mode(FrozenTarget, ("symbolId", "addressId")) == 2
    assert smx_host_ctor_mode(PostOp, names) == 0
    assert smx_host_ctor_mode(PlainOp, names) == 0
    assert smx_host_ctor_mode(Target, ("addressId", "symbolId")) == 0

    def mk(cls, tcls, i, typ, ts, **p):
        return cls(f"i{i}", 1, typ, tcls(f"s{i % 2}", "a"), p, {}, {}, {"timestamp": ts})
    A = [mk(PostOp, FrozenTarget, 0, "moveDecl", "t1", newAddress="x"),
         mk(PlainOp, Target, 1, "editStmtBlock", "t2")]
    B = [mk(PostOp, Target, 2, "editStmtBlock", "t3"), mk(PlainOp, FrozenTarget, 3, "moveDecl", "t0", newFile="f")]
    PostOp.calls = 0
    out, _ = _native(A, B)
    assert PostOp.calls == 4  # two inputs, one clone each in native and in Python
    assert {type(o.target) for o in out} == {FrozenTarget, Target}


def test_errors_propagate():
    bad = _op("editStmtBlock", "s1")
    del bad.provenance
    with pytest.raises(AttributeError):
        marshal_native([bad], [])

    class Unhashable(list):
        pass
    with pytest.raises(TypeError):
        marshal_native([_op(Unhashable(), "s1")], [])


def test_empty():
    soa = marshal_native([], [])
    _soa_equal(soa, marshal([], []))
    assert materialize_ops_native([], soa.kind, soa.strings, *([np.zeros(0, np.int32)] * 4)) == []
