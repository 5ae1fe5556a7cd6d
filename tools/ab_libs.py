"""A/B timing of several libsmx builds in ONE process (interleaved rounds, same inputs,
same clock state; cdna_hip_programming.md §5.4 rule 24):

    python tools/ab_libs.py [--config c3] [--n-ops N] [--rounds 5] [--verify] name=path ...

Each build is loaded under its own path (its own globals).  Per round and build: one
warm-up merge, then 3 merges with the library's per-stage HIP events; prints the median
per-stage ms per merge.  --verify checks each build's outputs against the C oracle
once (small configs only)."""
import argparse
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--n-ops", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--verify", action="store_true")
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    import torch
    from semantic_merge_amd import _abi, _lib, synth
    spec = synth.CONFIGS[a.config]
    if a.n_ops:
        spec = synth.LiftSpec(**{**spec.__dict__, "n_total": a.n_ops})
    soa = synth.lift_soa(synth.lift_logs(spec))
    dc = _lib.DeviceCompose(soa)
    libs = []
    for item in a.libs:
        name, path = item.split("=", 1)
        libs.append((name, _abi.declare(C.CDLL(os.path.abspath(path)))))
    # one workspace large enough for every build (their layouts may differ)
    need = 0
    for _, L in libs:
        ws = C.c_size_t(0)
        assert L.smx_compose_workspace_bytes(soa.n_a, soa.n_b, soa.n_sym, C.byref(ws)) == 0
        need = max(need, ws.value)
    if need > dc.ws_bytes:
        dc.ws = torch.empty(need, dtype=torch.uint8, device=dc.device)
        dc.ws_bytes = need
    ref = None
    if a.verify:
        from oracle import oracle
        ref = oracle.compose(soa)

    def stages(L):
        ms = (C.c_double * 16)()
        calls = (C.c_int64 * 16)()
        n = L.smx_stage_times(ms, calls, 16)
        return {L.smx_stage_name(i).decode(): (ms[i], calls[i]) for i in range(n)}

    res = {name: {} for name, _ in libs}
    for rnd in range(a.rounds):
        for name, L in libs:
            rc = L.smx_compose(*dc._args(None))
            assert rc == 0, (name, L.smx_last_error())
            torch.cuda.synchronize()
            if rnd == 0 and ref is not None:
                got = dc.results()
                ok = all(np.array_equal(g, r) for g, r in zip(got, ref))
                print(f"{name}: verify {'OK' if ok else 'MISMATCH'}", flush=True)
                if not ok:
                    sys.exit(3)
            L.smx_reset_stage_times()
            L.smx_set_profiling(1)
            for _ in range(3):
                L.smx_compose(*dc._args(None))
            torch.cuda.synchronize()
            L.smx_set_profiling(0)
            for k, (ms, c) in stages(L).items():
                if c:
                    res[name].setdefault(k, []).append(ms / 3)
    for name, _ in libs:
        r = res[name]
        tot = sum(np.median(v) for k, v in r.items() if k != "segsort")  # (segsort lies inside gsort)
        print(f"{name:12s} " + "  ".join(f"{k} {np.median(v):.3f}" for k, v in r.items())
              + f"  | total {tot:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
