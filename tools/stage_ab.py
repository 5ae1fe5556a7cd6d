"""A/B timing of the compose stages for one library build (SMX_LIB=...):
median over rounds of per-stage ms per merge (all calls of a stage in one merge summed,
e.g. failed presorted attempts before the generic plan) on the c3 workload (or
argv[1] ops of config argv[2], argv[3] symbols)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    from semantic_merge_amd import _lib, synth
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    cfg = sys.argv[2] if len(sys.argv) > 2 else "c3"
    kw = {"n_total": n}
    if len(sys.argv) > 3:
        kw["n_sym"] = int(sys.argv[3])
    spec = synth.LiftSpec(**{**synth.CONFIGS[cfg].__dict__, **kw})
    soa = synth.lift_soa(synth.lift_logs(spec))
    dc = _lib.DeviceCompose(soa)
    lib = _lib.lib()
    for _ in range(2):
        dc.run()
    torch.cuda.synchronize()
    res = {}
    runs = 3
    for _ in range(5):
        lib.smx_reset_stage_times()
        lib.smx_set_profiling(1)
        for _ in range(runs):
            dc.run()
        torch.cuda.synchronize()
        lib.smx_set_profiling(0)
        for k, (ms, c) in _lib.stage_times().items():
            if c:
                res.setdefault(k, []).append(ms / runs)
    tot = sum(np.median(v) for k, v in res.items() if k != "segsort")  # (segsort lies inside gsort)
    print("  ".join(f"{k} {np.median(v):.3f}" for k, v in res.items()) + f"  | total {tot:.3f} ms")


if __name__ == "__main__":
    main()
