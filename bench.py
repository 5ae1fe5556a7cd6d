"""Benchmark: op-log compose+conflict throughput on device-resident synthetic logs.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3] [--n-ops N]

One step = one composition (semmerge/compose.py:11-114 restated on the GPU) of
SURVEY §8(d) config 3: 100M lift-shaped ops (50M per branch) per GPU, 1M symbols,
seed 11.  Inputs are resident in HBM before timing.  N = 1: one smx_compose call.
N > 1 (torchrun, one process per GPU): ONE merge of N x 100M ops sharded by
timestamp key range (semantic_merge_amd/shard.py): each rank starts from its
index slices of both branch logs, and a step is the whole sharded composition --
the RCCL all-to-all that moves ops to their key-range shard, the per-shard
kernels, the walk hand-off and the MAX all-reduce of the chain tables (weak
scaling: 100M ops per GPU).  --independent runs N unrelated merges instead.  The
time is the max over ranks; rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "op-log compose+conflict throughput (ops/s), 100M-op logs, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
PIPE_BYTES_PER_OP = 53         # 37 B in + 16 B out per op (+8 B per conflict)
WINDOW_BYTES_PER_OP = 41       # k_window: 37 B of input read once + 4 B T-order index written


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--n-ops", type=int, default=0, help="override the config's op count")
    ap.add_argument("--n-sym", type=int, default=0, help="override the config's symbol count")
    ap.add_argument("--cpu-sample", type=int, default=40_000_000,
                    help="ops in the CPU-baseline sample (rank 0, N=1 only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify", action="store_true", help="check GPU == oracle (slow, N = 1)")
    ap.add_argument("--independent", action="store_true",
                    help="N > 1: independent merges per rank instead of one sharded merge")
    args = ap.parse_args()

    import torch
    from semantic_merge_amd import _lib, synth
    from semantic_merge_amd.dist import job_throughput, max_over_ranks, rank_info, rank_seed

    ri = rank_info()
    world, rank, local = ri.world, ri.rank, ri.local
    dist = None
    # SMX_BENCH_BACKEND=gloo: rehearse N ranks on fewer GPUs (collectives through host
    # copies); the driver's multi-GPU runs use RCCL, one GPU per rank.
    backend = os.environ.get("SMX_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(torch.cuda.device_count(), 1)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)

    spec = synth.CONFIGS[args.config]
    if args.n_ops:
        spec = synth.LiftSpec(**{**spec.__dict__, "n_total": args.n_ops})
    if args.n_sym:
        spec = synth.LiftSpec(**{**spec.__dict__, "n_sym": args.n_sym})
    sharded = world > 1 and not args.independent
    t0 = time.time()
    sc = dc = None
    if sharded:
        from semantic_merge_amd import shard
        soa, na_g, nb_g = synth.lift_slice_soa(spec, rank, world)
        sl_a, sl_b, _, _ = shard.slices_from_soa(soa, 0, 1, dev)
        log(f"[rank {rank}] generated slice of {soa.n:,} ops in {time.time() - t0:.1f}s")
        sc = shard.ShardedCompose(sl_a, sl_b, na_g, nb_g, soa.n_sym, shard.Comm(), dev)
        del sl_a, sl_b
        run = sc.run
        log(f"[rank {rank}] resident on {dev}; shard buffers with headroom {sc.hd:,}")
    else:
        spec = synth.LiftSpec(**{**spec.__dict__, "seed": rank_seed(spec.seed, rank)})
        logs = synth.lift_logs(spec)
        soa = synth.lift_soa(logs)
        del logs
        log(f"[rank {rank}] generated {soa.n:,} ops in {time.time() - t0:.1f}s")
        dc = _lib.DeviceCompose(soa, f"cuda:{local}")
        run = dc.run
        log(f"[rank {rank}] resident on {dev}; workspace {dc.ws_bytes / 2**30:.2f} GiB")

    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize(dev)

    lib = _lib.lib()
    lib.smx_reset_stage_times()
    lib.smx_set_profiling(1)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    lib.smx_set_profiling(0)
    stages = _lib.stage_times()
    if sharded:
        fin = sc.sum_final
        nconf = int(fin[:, shard.S_NCONF].sum())
        k = world * soa.n - int(fin[:, shard.S_NSKIP].sum())
    else:
        k, nconf = (int(x) for x in dc.counts.cpu().tolist())
    elapsed = max_over_ranks(elapsed, dev)

    if args.verify and not sharded:
        from oracle import oracle
        ref = oracle.compose(soa)
        got = dc.results()
        ok = all(np.array_equal(g, r) for g, r in zip(got, ref))
        log(f"[rank {rank}] verify vs oracle: {'OK' if ok else 'MISMATCH'}")
        if not ok:
            sys.exit(3)

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    n = soa.n
    ms_step = elapsed / args.steps * 1e3
    value = job_throughput(n, world, args.steps, elapsed)
    win_ms, win_calls = stages.get("window", (0.0, 0))
    win_avg = win_ms / max(win_calls, 1)
    achieved = WINDOW_BYTES_PER_OP * n / (win_avg * 1e-3) / 1e9 if win_avg > 0 else None
    traffic = None
    prof = os.path.join(REPO, "profiles", "pmc_window.json")
    if os.path.exists(prof) and args.config == "c3":  # measured on the config-3 window kernel
        rec = json.load(open(prof))
        if rec.get("n_ops") == n:
            traffic = rec.get("hbm_bytes_per_launch")
    pipe_gbs = (PIPE_BYTES_PER_OP * n + 8 * nconf) / (ms_step * 1e-3) / 1e9

    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        from oracle import oracle
        from semantic_merge_amd.marshal import SoA
        half = min(args.cpu_sample // 2, soa.n_a, soa.n_b)
        idx = np.concatenate([np.arange(half), soa.n_a + np.arange(half)])
        sample = SoA(half, half, soa.kind[idx], soa.ts[idx], soa.oid_hi[idx], soa.oid_lo[idx],
                     soa.sym[idx], soa.v0[idx], soa.v1[idx], soa.n_sym)
        t0 = time.perf_counter()
        oracle.compose(sample)
        dt = time.perf_counter() - t0
        cpu = {"value": round(2 * half / dt, 1), "unit": "ops/s", "cores": 1, "kind": "port",
               "sample": f"first {half:,} ops of each branch of the same workload "
                         f"({2 * half:,} ops) through oracle/compose_ref.c, 1 thread, "
                         f"{dt:.1f}s"}

    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "ops/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (lift-shaped op logs generated from a seed, SURVEY §8(d))",
        "config": {
            "workload": (f"{args.config}: one merge of {world * n:,} ops ({n:,} per GPU, "
                         f"{soa.n_a:,} per branch per GPU), {soa.n_sym:,} symbols, "
                         f"{spec.ops_per_ms} ops/ms, seed {spec.seed}"
                         + (", sharded by timestamp key range" if sharded else "")
                         + (f", {world} independent merges" if world > 1 and not sharded else "")),
            "n_ops_per_gpu": n,
            "n_ops_total": world * n,
            "n_sym": soa.n_sym,
            "composed_ops": k,
            "conflicts": nconf,
            "parallelism": (f"key-range shards x{world} (RCCL all-to-all + all-gathers + "
                            f"MAX all-reduce)" if sharded else
                            (f"independent merges x{world}" if world > 1 else "single GPU")),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "k_window",
            "achieved": round(achieved, 1) if achieved else None,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
            "traffic": traffic,
            "bytes_per_op": WINDOW_BYTES_PER_OP,
            "avg_launch_ms": round(win_avg, 4),
        },
        "pipeline_roofline": {
            "bytes_per_op": PIPE_BYTES_PER_OP,
            "achieved": round(pipe_gbs, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(pipe_gbs / HBM_PEAK_GBS, 4),
        },
        "stages_ms_per_step": {k2: round(v[0] / max(v[1], 1), 4) for k2, v in stages.items()
                               if v[1]},
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
