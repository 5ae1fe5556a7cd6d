"""Graph-replay check (diagnostics): the same buffers composed with new inputs, merge by
merge against the oracle; prints which merge differs."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from oracle import oracle
    from semantic_merge_amd import _lib, synth
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 600_000
    soas = [synth.lift_soa(synth.lift_logs(synth.LiftSpec(n, 4_000, sd))) for sd in (31, 32, 33)]
    dc = _lib.DeviceCompose(soas[0])
    s = torch.cuda.Stream()
    for rep, soa in enumerate(soas + soas[:1]):
        for name, col, dt in (("kind", soa.kind, np.uint8), ("ts", soa.ts, np.int64), ("hi", soa.oid_hi, np.int64),
                              ("lo", soa.oid_lo, np.int64), ("sym", soa.sym, np.int32), ("v0", soa.v0, np.int32),
                              ("v1", soa.v1, np.int32)):
            getattr(dc, name).copy_(torch.from_numpy(np.ascontiguousarray(col).view(dt)))
        torch.cuda.synchronize()
        try:
            dc.run(s)
            s.synchronize()
            got = dc.results()
            ref = oracle.compose(soa)
            ok = [bool(np.array_equal(g, r)) for g, r in zip(got, ref)]
            print(f"merge {rep}: {ok} counts {dc.counts.cpu().tolist()}", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"merge {rep}: error {e}", flush=True)
            meta = dc.ws[:256].cpu().numpy().view(np.uint64)
            print("   meta words", meta[:48].tolist(), flush=True)


if __name__ == "__main__":
    main()
