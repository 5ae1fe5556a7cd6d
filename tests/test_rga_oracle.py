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
