"""The pure-Python restatement (oracle/compose_ref.py, bench.py's single-core Python
leg) agrees with the C oracle and with the reference's own golden outputs."""
import numpy as np

from oracle import compose_ref, oracle
from semantic_merge_amd import synth

from _util import assert_case, load


def test_python_restatement_matches_reference_golden():
    for name, case in load("compose_scenarios.json").items():
        assert_case(compose_ref.compose, case, name)
    for i, case in enumerate(load("compose_cases.json")[:200]):
        assert_case(compose_ref.compose, case, f"case {i}")


def test_python_restatement_matches_c_oracle():
    for cfg in ("c2", "c5"):
        spec = synth.LiftSpec(**{**synth.CONFIGS[cfg].__dict__, "n_total": 40_000})
        soa = synth.lift_soa(synth.lift_logs(spec))
        got, ref = compose_ref.compose(soa), oracle.compose(soa)
        for g, r in zip(got, ref):
            assert np.array_equal(g, r), cfg
