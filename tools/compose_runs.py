"""Minimal driver for counter passes: K merges of the config-3 workload (or argv[2] ops;
COMPOSE_CFG=c5 for config 5's shape)
through DeviceCompose, no checks (SMX_ABLATE runs produce invalid results by design)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    from semantic_merge_amd import _lib, synth
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000_000
    cfg = os.environ.get("COMPOSE_CFG", "c3")  # (c5: config 5's shape at n ops)
    spec = synth.LiftSpec(**{**synth.CONFIGS[cfg].__dict__, "n_total": n})
    dc = _lib.DeviceCompose(synth.lift_soa(synth.lift_logs(spec)))
    for _ in range(k):
        dc.run()
    torch.cuda.synchronize()
    print("done", k)


if __name__ == "__main__":
    main()
