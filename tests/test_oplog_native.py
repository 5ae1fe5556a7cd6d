"""Native Op.from_dict (semantic_merge_amd.oplog, csrc/smx_host.cpp) against the Python
restatement of ops.py:89-100 on the golden inputs and on coercion / error corners. CPU only."""
import dataclasses
import json
from collections import OrderedDict
from typing import Any, Optional

import pytest

from semantic_merge_amd import synth
from semantic_merge_amd.oplog import oplog_from_json, ops_from_dicts, ops_from_worker_result
from semantic_merge_amd.ops import Op, Target

from _util import jline, load


def _same(got, ref):
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        assert type(g) is type(r) and type(g.target) is type(r.target)
        assert g == r
        assert jline(g.to_dict()) == jline(r.to_dict())
        for f in ("params", "guards", "effects", "provenance"):
            assert type(getattr(g, f)) is dict


def test_golden_inputs():
    items = []
    for case in load("compose_cases.json")[:200]:
        items += case["A"] + case["B"]
    got = ops_from_dicts(items)
    _same(got, [Op.from_dict(d) for d in items])
    for g, d in zip(got, items):  # fresh top-level dicts, shared nested values (dict(x) is shallow)
        assert g.params is not d.get("params")


def test_synthetic_and_json_and_worker_result():
    A, B = synth.lift_op_dicts(synth.lift_logs(synth.LiftSpec(20_000, 500, 5)))
    text = json.dumps(A)
    _same(oplog_from_json(text), [Op.from_dict(d) for d in json.loads(text)])
    left, right, maps = ops_from_worker_result({"opLogLeft": A, "opLogRight": B, "symbolMaps": {"x": 1}})
    _same(left, [Op.from_dict(d) for d in A])
    _same(right, [Op.from_dict(d) for d in B])
    assert maps == {"x": 1}
    assert ops_from_worker_result({}) == ([], [], {})


def test_coercions():
    items = [
        {"id": 7, "type": "renameSymbol", "target": {"symbolId": "s", "addressId": None}},
        {"id": "x", "schemaVersion": "3", "type": 5, "target": {"symbolId": "s"},
         "params": [("a", 1)], "guards": OrderedDict(g=1), "provenance": {"timestamp": 1.5}},
        {"id": 1.25, "schemaVersion": 2.9, "type": None, "target": {"addressId": "a", "symbolId": "s"},
         "effects": {}},
        OrderedDict(id="m", type="t", target={"symbolId": "q", "addressId": "r"}, params={"k": [1]}),
    ]
    _same(ops_from_dicts(items), [Op.from_dict(d) for d in items])


class GetLogger(dict):
    calls = []

    def get(self, key, default=None):
        GetLogger.calls.append(key)
        return super().get(key, default)


def test_mapping_get_is_called_like_the_reference():
    d = GetLogger(id="a", type="t", target={"symbolId": "s", "addressId": None}, params={"p": 1})
    GetLogger.calls = []
    got = ops_from_dicts([d])
    native_calls = list(GetLogger.calls)
    GetLogger.calls = []
    ref = [Op.from_dict(d)]
    assert native_calls == GetLogger.calls
    _same(got, ref)


@pytest.mark.parametrize("bad, exc", [
    ({"type": "t", "target": {"symbolId": "s"}}, KeyError),                        # no id
    ({"id": "a", "target": {"symbolId": "s"}}, KeyError),                          # no type
    ({"id": "a", "type": "t"}, KeyError),                                          # no target
    ({"id": "a", "type": "t", "target": {"symbolId": "s", "x": 1}}, TypeError),    # unknown field
    ({"id": "a", "type": "t", "target": 5}, TypeError),                            # ** of a non-mapping
    ({"id": "a", "type": "t", "target": {"symbolId": "s"}, "params": None}, TypeError),
    ({"id": "a", "type": "t", "target": {"symbolId": "s"}, "schemaVersion": "v1"}, ValueError),
])
def test_errors_match(bad, exc):
    with pytest.raises(exc):
        Op.from_dict(bad)
    with pytest.raises(exc):
        ops_from_dicts([bad])


@dataclasses.dataclass
class RefTarget:
    symbolId: str
    addressId: Optional[str] = None


@dataclasses.dataclass
class RefOp:
    id: str
    schemaVersion: int
    type: str
    target: RefTarget
    params: Any
    guards: Any
    effects: Any
    provenance: Any


class CountingTarget:
    made = 0

    def __init__(self, symbolId, addressId=None):
        CountingTarget.made += 1
        self.symbolId, self.addressId = symbolId, addressId


def test_other_classes():
    items = load("compose_cases.json")[0]["A"]
    got = ops_from_dicts(items, RefOp, RefTarget)
    assert all(type(o) is RefOp and type(o.target) is RefTarget for o in got)
    assert [dataclasses.asdict(o) for o in got] == [dataclasses.asdict(Op.from_dict(d)) for d in items]
    CountingTarget.made = 0
    got = ops_from_dicts(items, RefOp, CountingTarget)
    assert CountingTarget.made == len(items)
    assert [o.target.symbolId for o in got] == [d["target"]["symbolId"] for d in items]
