"""OpLog (semmerge/ops.py:106-121) on the native decoder: from_json decodes every
golden text exactly as the reference did (tools/make_golden.py ran the reference's own
OpLog.from_json), malformed ops raise the reference's exception class, and to_json
follows orjson's output rules (compact, non-ASCII kept, NaN -> null, str keys only,
64-bit integers)."""
import json
import math

import pytest

from semantic_merge_amd.oplog import OpLog, dumps, loads, oplog_from_json
from semantic_merge_amd.ops import Op

from _util import load

ERRORS = {"KeyError": KeyError, "TypeError": TypeError, "ValueError": ValueError}


def test_from_json_matches_reference_golden():
    cases = load("oplog_cases.json")
    assert len(cases) == 300
    n_err = 0
    for i, case in enumerate(cases):
        if "error" in case:
            n_err += 1
            with pytest.raises(ERRORS[case["error"]]):
                OpLog.from_json(case["text"])
            continue
        log = OpLog.from_json(case["text"])
        assert [o.to_dict() for o in log.ops] == case["ops"], f"case {i}"
        assert [o.to_dict() for o in oplog_from_json(case["text"].encode())] == case["ops"]
    assert n_err >= 20


def test_to_json_round_trip_and_format():
    for case in load("oplog_cases.json")[:120]:
        if "error" in case:
            continue
        log = OpLog.from_json(case["text"])
        text = log.to_json()
        assert json.loads(text) == case["ops"]
        assert text == json.dumps(case["ops"], separators=(",", ":"), ensure_ascii=False)
        again = OpLog.from_json(text)
        assert [o.to_dict() for o in again.ops] == case["ops"]


def test_orjson_rules():
    assert dumps([1.5, math.nan, math.inf, "é"]) == '[1.5,null,null,"é"]'
    with pytest.raises(TypeError):
        dumps({1: "x"})
    with pytest.raises(TypeError):
        dumps([2 ** 64])
    assert dumps([2 ** 64 - 1, -(2 ** 63)]) == f"[{2 ** 64 - 1},{-(2 ** 63)}]"
    for bad in ("[NaN]", "[Infinity]", "[-Infinity]"):
        with pytest.raises(ValueError):
            loads(bad)
    assert loads(b'[{"a":1}]') == [{"a": 1}]
    log = OpLog()
    log.extend([Op.from_dict({"id": "x", "type": "addDecl", "target": {"symbolId": "s"}})])
    assert OpLog.from_json(log.to_json()).ops == log.ops
