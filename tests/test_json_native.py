"""The native JSON reader and the one-pass OpLog decode (csrc/smx_host.cpp JsonReader,
decode_oplogs): the reader returns what the json module returns under orjson's input
rules, and decode_pair gives OpLog.from_json's ops (pinned by the reference fixtures)
together with exactly the SoA that marshal_native builds from them."""
import json
import math
import random

import numpy as np
import pytest

from semantic_merge_amd import synth
from semantic_merge_amd._host import host
from semantic_merge_amd.marshal import marshal_native
from semantic_merge_amd.oplog import OpLog, decode_pair, loads

from _util import load


def _rand_doc(rng, depth=0):
    r = rng.random()
    if depth > 4 or r < 0.45:
        return rng.choice([None, True, False, 0, -1, 7, 2 ** 70, -(2 ** 65), 1.5, -2.5e-8, 1e300, 0.1,
                           "", "a", "é", "☃", "\U0001f600", "\\", "\"q\"", "\n\t\u0001", "/", "\ud7ff"])
    if r < 0.7:
        return [_rand_doc(rng, depth + 1) for _ in range(rng.randint(0, 4))]
    return {rng.choice(["a", "b", "ключ", "k" * 20, "", "x\u2028"]): _rand_doc(rng, depth + 1)
            for _ in range(rng.randint(0, 4))}


def test_reader_matches_json_module():
    rng = random.Random(5)
    for i in range(2000):
        doc = _rand_doc(rng)
        for text in (json.dumps(doc), json.dumps(doc, ensure_ascii=False), json.dumps(doc, indent=2)):
            assert host().json_loads(text) == json.loads(text), text
            assert host().json_loads(text.encode()) == json.loads(text)
    for text in ('"\\ud83d\\ude00"', '[1e400, -1e400, 1E2, -0, -0.0]',
                 '{"a": 1, "a": 2}', ' \n[ ] ', '123456789012345678901234567890'):
        got, want = host().json_loads(text), json.loads(text)
        assert repr(got) == repr(want), text


@pytest.mark.parametrize("bad", ["[NaN]", "[Infinity]", "[-Infinity]", "[1,]", "{\"a\" 1}", "[1] x", "",
                                 "\"a\u0001\"", "[01]", "[1.]", "[.5]", "tru", "{'a': 1}", "[\"\\x\"]",
                                 "[" * 1100 + "]" * 1100, '"\\ud800"', '"\\udc00x"', '["\\ud83dx"]',
                                 b'["\xff"]', b'"\xed\xa0\x80"', "\"\ud800\""])
def test_reader_rejects(bad):
    """orjson's input rules (ops.py:117), raised as json.JSONDecodeError as orjson does
    (orjson.JSONDecodeError subclasses it): NaN / Infinity, lone surrogates (escaped or in
    the text), invalid UTF-8, nesting beyond 1024, trailing data."""
    if not isinstance(bad, bytes) and "\ud800" not in bad:
        with pytest.raises(json.JSONDecodeError):
            host().json_loads(bad)
    with pytest.raises(json.JSONDecodeError):
        loads(bad)


def test_decode_pair_error_order():
    """The reference parses a whole text before building any op (orjson.loads, then
    Op.from_dict per item): a syntax error late in the text wins over a bad item early;
    a bad item (KeyError) is raised when the text parses; the outer array counts toward
    the 1024 nesting limit."""
    good = json.dumps([{"id": "x", "type": "addDecl", "target": {"symbolId": "s"}}])
    bad_item = '[{"type": "addDecl"}, {"id": "y", "type": "addDecl", "target": {"symbolId": "s"}}'
    with pytest.raises(json.JSONDecodeError):
        decode_pair(bad_item + ", tru]", good)
    with pytest.raises(KeyError):
        decode_pair(bad_item + "]", good)
    with pytest.raises(json.JSONDecodeError):       # text b's JSON error after text a's items
        decode_pair(good, "[1,")
    deep = "[" + "[" * 1024 + "]" * 1024 + "]"
    with pytest.raises(json.JSONDecodeError):
        host().json_loads(deep)
    with pytest.raises(json.JSONDecodeError):
        decode_pair(deep, good)


def _soa_equal(a, b):
    for f in ("kind", "ts", "oid_hi", "oid_lo", "sym", "v0", "v1"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f
    assert (a.n_a, a.n_b, a.n_sym, a.strings, a.ts_mode, a.id_mode) == \
        (b.n_a, b.n_b, b.n_sym, b.strings, b.ts_mode, b.id_mode)


def test_decode_pair_matches_from_json_and_marshal():
    cases = load("oplog_cases.json")
    good = [c for c in cases if "error" not in c]
    bad = [c for c in cases if "error" in c]
    for x, y in zip(good[::2], good[1::2]):
        ops_a, ops_b, soa = decode_pair(x["text"], y["text"])
        assert [o.to_dict() for o in ops_a] == x["ops"] and [o.to_dict() for o in ops_b] == y["ops"]
        _soa_equal(soa, marshal_native(ops_a, ops_b))
    errs = {"KeyError": KeyError, "TypeError": TypeError, "ValueError": ValueError}
    for c in bad:
        with pytest.raises(errs[c["error"]]):
            decode_pair(good[0]["text"], c["text"])


def test_decode_pair_lift_logs():
    logs = synth.lift_logs(synth.LiftSpec(20_000, 300, 4))
    A, B = synth.lift_op_dicts(logs)
    ta, tb = json.dumps(A), json.dumps(B).encode()
    ops_a, ops_b, soa = decode_pair(ta, tb)
    ref_a, ref_b = OpLog.from_json(ta).ops, OpLog.from_json(tb).ops
    assert ops_a == ref_a and ops_b == ref_b
    _soa_equal(soa, marshal_native(ref_a, ref_b))
    # a document that is not a list is iterated like the reference's comprehension
    with pytest.raises(TypeError):
        decode_pair('{"id": 1}', "[]")
    assert math.isinf(host().json_loads("1e999"))
