"""Fixed costs of the sharded step (semantic_merge_amd/shard.py) on one GPU: a one-rank
RCCL ("nccl") group runs ShardedCompose on the slice one rank of an N-way strong split
of config 3 holds, next to the plain smx_compose of the same ops.  The difference is
what the sharded machinery adds per step before any cross-GPU traffic (host syncs,
collectives, extra launches).  Diagnostics only.

    python tools/shard_probe.py [N ...]      (default 1 2 4 8)
"""
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from semantic_merge_amd import _lib, shard, synth  # noqa: E402


def timed(fn, steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def breakdown(sc, steps=5):
    """Per-phase ms of ShardedCompose.run with a device sync around each phase (the syncs
    add their own cost; the phases' relative weights are what this shows)."""
    import collections
    acc = collections.defaultdict(float)
    names = {v: k for k, v in vars(shard._abi).items() if k.startswith("SHARD_") and isinstance(v, int)}

    def wrap(name, fn):
        def w(*a, **k):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = fn(*a, **k)
            torch.cuda.synchronize()
            key = name if name != "_step" else "step:" + names.get(a[0], str(a[0]))
            acc[key] += (time.perf_counter() - t0) * 1e3
            return r
        return w
    saved = {}
    for m in ("exchange", "_order_exchange", "_walk", "_step", "_bind"):
        saved[m] = getattr(sc, m)
        setattr(sc, m, wrap(m, saved[m]))
    saved_ar = sc.comm.all_reduce_max
    sc.comm.all_reduce_max = wrap("all_reduce_max", saved_ar)
    for _ in range(steps):
        sc.run()
    for m, f in saved.items():
        setattr(sc, m, f)
    sc.comm.all_reduce_max = saved_ar
    return {k: round(v / steps, 3) for k, v in acc.items()}


def main():
    ns = [int(x) for x in sys.argv[1:]] or [1, 2, 4, 8]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    dev = torch.device("cuda", 0)
    base = synth.CONFIGS["c3"]
    for n in ns:
        spec = synth.LiftSpec(**{**base.__dict__, "n_total": base.n_total // n})
        soa, na_g, nb_g = synth.lift_slice_soa(spec, 0, n)
        dc = _lib.DeviceCompose(soa, "cuda:0")
        for _ in range(2):
            dc.run()
        plain = timed(dc.run, 10)
        del dc
        a, b, _, _ = shard.slices_from_soa(soa, 0, 1, dev)
        sc = shard.ShardedCompose(a, b, soa.n_a, soa.n_b, soa.n_sym, shard.Comm(), dev, mode="range")
        for _ in range(2):
            sc.run()
        sh = timed(sc.run, 10)
        print(f"N={n}: {soa.n:,} ops per rank: plain smx_compose {plain:.3f} ms, one-rank sharded step "
              f"{sh:.3f} ms (+{sh - plain:.3f})", flush=True)
        print(f"   phases (synced): {breakdown(sc)}", flush=True)
        if os.environ.get("SHARD_PROBE_PROFILE"):  # host-side hot spots of the step (cProfile)
            import cProfile
            import pstats
            pr = cProfile.Profile()
            pr.enable()
            for _ in range(20):
                sc.run()
            torch.cuda.synchronize()
            pr.disable()
            pstats.Stats(pr).sort_stats("tottime").print_stats(30)
            pstats.Stats(pr).sort_stats("cumtime").print_stats(40)
        del sc, a, b, soa
        torch.cuda.empty_cache()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
