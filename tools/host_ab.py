"""A/B of native host modules (_smx_host.so builds) in ONE process, alternating:
materialise (100k-op config-2 log in output order, and a 1k-op one) and marshal.

    python tools/host_ab.py name=path/_smx_host.so ...
"""
import importlib.util
import os
import sys
import time
from copy import deepcopy

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def load(name, path):
    spec = importlib.util.spec_from_file_location("_smx_host", path)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def main():
    from oracle import oracle
    from semantic_merge_amd import synth
    from semantic_merge_amd.marshal import marshal_native
    from semantic_merge_amd.materialize import KIND_MOVE, KIND_RENAME, smx_host_ctor_mode
    from semantic_merge_amd.oplog import ops_from_dicts
    mods = [(a.split("=", 1)[0], load(*a.split("=", 1))) for a in sys.argv[1:]]
    i32 = lambda a: np.ascontiguousarray(a, dtype=np.int32)
    cases = []
    for n in (100000, 1000):
        logs = synth.lift_logs(synth.LiftSpec(n, max(n // 100, 10), 7))
        A, B = synth.lift_op_dicts(logs)
        oa, ob = ops_from_dicts(A), ops_from_dicts(B)
        soa = marshal_native(oa, ob)
        order, addr, file, ctx, _ = oracle.compose(soa)
        cases.append((n, oa, ob, soa, (i32(order), i32(addr), i32(file), i32(ctx))))
    res = {}
    for rnd in range(9):
        for name, m in mods:
            for n, oa, ob, soa, (o, a, f, c) in cases:
                reps = 1 if n >= 100000 else 50
                ops = oa + ob
                t0 = time.perf_counter()
                for _ in range(reps):
                    out = m.materialize_ops(ops, np.ascontiguousarray(soa.kind, dtype=np.uint8), list(soa.strings),
                                            o, a, f, c, KIND_MOVE, KIND_RENAME, deepcopy, smx_host_ctor_mode)
                t1 = time.perf_counter()
                del out
                res.setdefault((name, n, "materialize"), []).append((t1 - t0) / reps)
    for (name, n, leg), v in sorted(res.items()):
        print(f"{name:10s} n={n:7d} {leg:12s} median {np.median(v) * 1e3:9.3f} ms  min {min(v) * 1e3:9.3f} ms", flush=True)


if __name__ == "__main__":
    main()
