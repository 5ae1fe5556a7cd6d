"""Latency of small merges (the CLI's real sizes: thousands of ops, and config 2).

    python tools/small_merge_probe.py [--sizes 1000,10000,100000,1000000] [--reps 50]

Per size, the median over --reps merges of:
  session_ms   compose_soa (the drop-in's device leg): pinned host pack, one host->device
               copy, smx_compose, one device->host copy, one sync -- sizes differ per call
               in real use, so the buffers are laid out per size (no graph replay)
  device_ms    DeviceCompose.run on resident buffers (smx_compose + its sync), repeated
               on the same buffers (the library replays its graph from the second call)
Prints one JSON line.  Run under rocprofv3 --kernel-trace for the launch timeline.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1000,10000,100000,1000000")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--verify", action="store_true")
    a = ap.parse_args()
    import torch
    from semantic_merge_amd import _lib, synth
    out = {}
    for n in [int(x) for x in a.sizes.split(",")]:
        spec = synth.LiftSpec(**{**synth.CONFIGS["c2"].__dict__, "n_total": n, "n_sym": max(n // 100, 10)})
        soa = synth.lift_soa(synth.lift_logs(spec))
        if a.verify:
            from oracle import oracle
            ref = oracle.compose(soa)
            got = _lib.compose_soa(soa)
            assert all(np.array_equal(g, r) for g, r in zip(got, ref)), n
        for _ in range(3):
            _lib.compose_soa(soa)
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            _lib.compose_soa(soa)
            ts.append(time.perf_counter() - t0)
        dc = _lib.DeviceCompose(soa)
        st = torch.cuda.Stream()
        for _ in range(3):
            dc.run(st)
        st.synchronize()
        td = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            dc.run(st)
            st.synchronize()
            td.append(time.perf_counter() - t0)
        out[n] = {"session_ms": round(float(np.median(ts)) * 1e3, 4), "device_ms": round(float(np.median(td)) * 1e3, 4),
                  "plan": _lib.DeviceCompose.last_plan()}
        print(n, out[n], file=sys.stderr, flush=True)
    print(json.dumps({"small_merges": out}))


if __name__ == "__main__":
    main()
