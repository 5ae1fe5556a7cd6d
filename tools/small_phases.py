"""Phase latencies of the one-workgroup small-merge kernel (smx_small.h), from the
wall-clock stamps of a -DSMALL_STAMPS build (tools/build_variants.sh stamps:"-DSMALL_STAMPS"):

    SMX_LIB=tools/_build/var_stamps/libsmx.so python tools/small_phases.py [--sizes 1000,2000]

Per size and log shape, the median over --reps calls of each phase (us).  Diagnostics only."""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES = ["load", "order check", "sort", "block bounds", "rename lists", "walk", "hash init",
          "slots", "chains + scan", "materialize"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1000,2000")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from semantic_merge_amd import _lib, synth
    lib = _lib.lib()
    lib.smx_diag_small_stamps.argtypes = [C.c_void_p]
    st = (C.c_uint64 * 16)()
    out = {}
    for n in [int(x) for x in a.sizes.split(",")]:
        for shape, spec in (("c2-like", synth.LiftSpec(n, max(n // 100, 10), 7)),
                            ("adversarial", synth.LiftSpec(n, max(n // 100, 10), 8, ops_per_ms=4096,
                                                           mix=synth.ADVERSARIAL_MIX, rename_overlap=1.0))):
            soa = synth.lift_soa(synth.lift_logs(spec))
            dc = _lib.DeviceCompose(soa)
            rows = []
            for _ in range(a.reps):
                dc.run()
                torch.cuda.synchronize()
                lib.smx_diag_small_stamps(st)
                v = np.array(list(st), dtype=np.float64)
                rows.append(np.diff(v[:11]) * 0.01)  # 100 MHz ticks -> us
            med = np.median(np.array(rows), axis=0)
            out[f"{n} {shape}"] = {"unordered": int(st[15]), "total_us": round(float(med.sum()), 2),
                                   **{p: round(float(x), 2) for p, x in zip(PHASES, med)}}
            print(f"{n} {shape}", out[f"{n} {shape}"], file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
