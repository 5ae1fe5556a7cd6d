"""Quick parity check of several libsmx builds (SMX_LIB per subprocess-free load):
    python tools/parity_libs.py name=path ...
Each build composes a few small lift logs; prints OK or the first differing output."""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch  # noqa: F401
    from oracle import oracle
    from semantic_merge_amd import _abi, _lib, synth
    specs = [synth.LiftSpec(n, s, seed) for n, s, seed in ((5000, 50, 1), (20_000, 200, 3), (300_000, 3000, 5))]
    specs += [synth.LiftSpec(600_000, 2_000, 17, ops_per_ms=4096, mix=synth.ADVERSARIAL_MIX),  # segmented plan
              synth.LiftSpec(300_000, 3_000, 7, shuffle=True)]                                 # radix plan
    cases = [synth.lift_soa(synth.lift_logs(sp)) for sp in specs]
    refs = [oracle.compose(c) for c in cases]
    for item in sys.argv[1:]:
        name, path = item.split("=", 1)
        L = _abi.declare(C.CDLL(os.path.abspath(path)))
        for c, ref in zip(cases, refs):
            dc = _lib.DeviceCompose(c)
            rc = L.smx_compose(*dc._args(None))
            torch.cuda.synchronize()
            got = dc.results()
            bad = [nm for nm, g, r in zip(("order", "addr", "file", "ctx", "conf"), got, ref)
                   if g.shape != r.shape or not np.array_equal(g, r)]
            print(f"{name} n={c.n}: rc={rc} {'OK' if not bad else 'MISMATCH ' + ','.join(bad)}", flush=True)


if __name__ == "__main__":
    main()
