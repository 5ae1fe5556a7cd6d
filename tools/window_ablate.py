"""Window-kernel ablation (diagnostic build, SMX_LIB=<-DSMX_DIAG=1 build>): time
k_window_f variants in ONE process, interleaved rounds (cdna_hip_programming.md §5.4
rule 24).  SMX_ABLATE = 16: load only; 100 + N: leave after phase N (smx_window.h
WF_EXIT), so phase N costs exitN - exit(N-1).  Results of ablated runs are invalid by
design; only the window stage time is read."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    from semantic_merge_amd import _lib, synth
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    spec = synth.LiftSpec(**{**synth.CONFIGS["c3"].__dict__, "n_total": n})
    soa = synth.lift_soa(synth.lift_logs(spec))
    dc = _lib.DeviceCompose(soa)
    lib = _lib.lib()
    names = {2: "merge", 3: "ksplit", 4: "kscan", 5: "kscatter", 6: "gbits", 7: "pkey", 8: "bucket",
             9: "renrank", 10: "posl", 11: "flags", 12: "out1"}
    variants = [("base", {}), ("loadonly", {"SMX_ABLATE": "16"})] + \
        [(f"exit{k:02d}_{v}", {"SMX_ABLATE": str(100 + k)}) for k, v in names.items()]
    res = {k: [] for k, _ in variants}
    for rnd in range(4):
        for name, env in variants:
            for k in ("SMX_ABLATE", "SMX_WIN_TGT"):
                os.environ.pop(k, None)
            os.environ.update(env)
            dc.run()
            torch.cuda.synchronize()
            lib.smx_reset_stage_times()
            lib.smx_set_profiling(1)
            for _ in range(5):
                dc.run()
            torch.cuda.synchronize()
            lib.smx_set_profiling(0)
            st = _lib.stage_times()
            ms, calls = st["window"]
            res[name].append(ms / max(calls, 1))
            tot = sum(v[0] for v in st.values()) / 5
            if rnd == 3:
                print(f"{name:10s} window {np.median(res[name]):.3f} ms  (min {min(res[name]):.3f})"
                      f"  all-stages {tot:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
