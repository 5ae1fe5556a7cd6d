"""Step-time probe on config 3: wall clock per smx_compose with and without the
per-stage HIP events, and the async (no host sync) variant.  Diagnostics only.

    python tools/timing_probe.py [--config c3] [--steps 20]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from semantic_merge_amd import _lib, synth  # noqa: E402


def timed(fn, steps, dev):
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    soa = synth.lift_soa(synth.lift_logs(synth.CONFIGS[a.config]))
    dc = _lib.DeviceCompose(soa, "cuda:0")
    lib = _lib.lib()
    for _ in range(3):
        dc.run()

    def run_async():
        dc.run_async()
        dc.finish()

    for rep in range(2):
        lib.smx_set_profiling(0)
        off = timed(dc.run, a.steps, dev)
        lib.smx_reset_stage_times()
        lib.smx_set_profiling(1)
        on = timed(dc.run, a.steps, dev)
        st = _lib.stage_times()
        lib.smx_set_profiling(0)
        asy = timed(run_async, a.steps, dev)
        stages = " ".join(f"{k} {v[0] / max(v[1], 1):.3f}" for k, v in st.items() if v[1])
        print(f"rep {rep}: events off {off:.3f} ms | events on {on:.3f} ms ({stages}) | async+finish {asy:.3f} ms",
              flush=True)


if __name__ == "__main__":
    main()
