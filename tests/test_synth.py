"""The numpy SoA generator is the exact image of marshalling its own Op rendering."""
import numpy as np

from semantic_merge_amd import synth
from semantic_merge_amd.marshal import marshal

from _util import to_ops


def _same_partition(a, b):
    """a and b induce the same equality classes (ids may be renumbered)."""
    pairs = set(zip(a.tolist(), b.tolist()))
    return len(pairs) == len(set(a.tolist())) == len(set(b.tolist()))


def test_soa_matches_marshalled_dicts():
    for spec in (synth.LiftSpec(6000, 40, 1), synth.LiftSpec(4000, 30, 2, shuffle=True),
                 synth.LiftSpec(5000, 20, 3, ops_per_ms=4096, mix=synth.ADVERSARIAL_MIX,
                                rename_overlap=0.3)):
        logs = synth.lift_logs(spec)
        soa = synth.lift_soa(logs)
        A, B = synth.lift_op_dicts(logs)
        m = marshal(to_ops(A), to_ops(B))
        for f in ("kind", "ts", "oid_hi", "oid_lo"):
            assert np.array_equal(getattr(m, f), getattr(soa, f)), f
        assert _same_partition(m.sym, soa.sym)
        for k in (0, 1):  # moves, renames: value ids equal up to renumbering
            sel = soa.kind == k
            assert np.array_equal(m.v0[sel] < 0, soa.v0[sel] < 0)
            assert _same_partition(m.v0[sel], soa.v0[sel]) and _same_partition(m.v1[sel], soa.v1[sel])


def test_iso_keys_vectorised_match_scalar():
    from semantic_merge_amd.marshal import iso_key
    ms = np.array([0, 999, 1000, 86_399_999, synth.BASE_MS, synth.BASE_MS + 123_456_789,
                   951_782_400_000, 4_102_444_800_000], dtype=np.int64)
    got = synth.iso_keys_from_ms(ms)
    for m, g in zip(ms.tolist(), got.tolist()):
        assert iso_key(synth.iso_string(m)) == g
