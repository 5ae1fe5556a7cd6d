"""Parity at BASELINE.json's full sizes: the GPU merge of config 3 (100M ops, 1M symbols)
and config 5 (20M adversarial ops) against digests of the C oracle's output, computed
off the box by tools/make_full_digest.py (tests/golden/full_digests.json).  The oracle
itself would take most of a minute at 100M ops; generating the logs takes about as long."""
import hashlib
import json
import os

import numpy as np
import pytest

from semantic_merge_amd import synth
from semantic_merge_amd._lib import compose_soa

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "full_digests.json")


def _digest(res) -> str:
    h = hashlib.sha256()
    for a in res:
        h.update(np.ascontiguousarray(a, dtype=np.int32).tobytes())
    return h.hexdigest()


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", ["c5", "c3"])
def test_full_size_digest(name):
    rec = {r["name"]: r for r in json.load(open(GOLDEN))}[name]
    soa = synth.lift_soa(synth.lift_logs(synth.CONFIGS[name]))
    assert soa.n == rec["n_ops"]
    res = compose_soa(soa, "cuda:0")
    del soa
    assert len(res[0]) == rec["n_out"] and len(res[4]) == rec["n_conflicts"]
    assert _digest(res) == rec["sha256"], f"{name}: GPU output differs from the oracle digest"
