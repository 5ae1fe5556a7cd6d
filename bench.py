"""Benchmark: op-log compose+conflict throughput on device-resident synthetic logs.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3] [--n-ops N]
                    [--weak | --independent] [--no-pmc] [--no-cpu-baseline] [--no-e2e] [--no-async] [--no-breakdown]

One step = one composition (semmerge/compose.py:11-114 restated on the GPU) of
SURVEY §8(d) config 3: 100M lift-shaped ops (50M per branch), 1M symbols, seed 11.
Inputs are resident in HBM before timing.  N = 1: one smx_compose call per step (on a
stream of its own, with the library's per-stage HIP events on: the roofline's kernel
time is measured inside the timed region; every step recomputes everything from the
inputs and syncs once).
N > 1 (torchrun, one process per GPU): by default ONE merge of the same 100M ops
split over the N ranks (strong scaling, BASELINE config 3 "100M ops across 8 GPUs"),
sharded by timestamp key range (semantic_merge_amd/shard.py); a step is the whole
sharded composition -- the packed all-to-all that moves ops to their key-range
shard, the per-shard kernels, the walk hand-off and the MAX all-reduce of the chain
tables.  --weak: N x 100M ops (100M per GPU); --independent: N unrelated merges.
The time is the max over ranks; rank 0 prints one JSON line.

roofline is SURVEY §8(d)'s figure for the whole merge: 53 B/op over the smx_compose
wall time (ms_per_step); kernel_roofline is the plan's dominant kernel alone.
Rank 0 at N = 1 also reports, after the timed steps (never inside them):
  roofline.traffic / kernel_roofline.traffic  HBM bytes per merge from rocprofv3 --pmc
        FETCH_SIZE and WRITE_SIZE passes over this same workload (child processes,
        one counter per pass; FETCH_SIZE x2 for gfx950's streaming reads, WRITE_SIZE
        x1, MI355X_MICROARCH.md "HBM"), null when rocprofv3 is unavailable
  cpu_baseline   the C port of the reference loop (oracle/compose_ref.c) on 1 thread,
        plus legs: the same on every host thread at once (independent samples),
        the pure-Python restatement (oracle/compose_ref.py) on 1 core, and the
        reference's own compose_oplogs as measured in the build container
  end_to_end     the drop-in compose_oplogs on a config-2-shaped log of Op objects:
        native marshal, device compose, native materialise
  small_merge    a 1k-op merge (the CLI's size): device latency on resident buffers (the
        one-workgroup plan) and the drop-in on Op objects
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "op-log compose+conflict throughput (ops/s), 100M-op logs, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
PIPE_BYTES_PER_OP = 53         # 37 B in + 16 B out per op (+8 B per conflict)
# The roofline kernel is the plan's dominant one, by the library's stage timers (the
# stage with the largest time per merge; its launches are averaged, so a stage holds one
# kernel instance -- the wide presorted windows have a stage of their own, apart from
# the normal attempt that failed before them):
#   stage        kernel (rocprof name prefix)  algorithmic bytes per op of the merge
#   window       k_window_f<2048              41: the 37 B of input read once + the 4 B T-order index
#   window_wide  k_window_f<8192              41: the same, 8192-op windows (config 5)
#   window_g     k_window_g                   45: the 37 B + the 4 B sort permutation + the 4 B index
#   segsort      k_segsort (2 launches)       52: ts, oid (24 B) read, sorted copies (24 B) + the
#                                             permutation (4 B) written
ROOF_STAGES = {"window": ("k_window_f<2048", 41), "window_wide": ("k_window_f<8192", 41),
               "window_g": ("k_window_g", 45), "segsort": ("k_segsort", 52)}
WINDOW_BYTES_PER_OP = ROOF_STAGES["window"][1]
ROOF_STEPS = 3  # timed steps whose roofline-kernel launches carry HIP events
REF_PY_OPS_S = 47_600          # SURVEY §3.4 / BASELINE.md: reference compose_oplogs, 1 core, 1M ops
FETCH_FACTOR, WRITE_FACTOR = 2.0, 1.0   # gfx950 FETCH_SIZE reads 1/2 of streamed bytes (guide)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pmc_traffic(args) -> dict:
    """HBM bytes per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over a
    child run of this benchmark (2 timed + 1 warm-up merges)."""
    exe = shutil.which("rocprofv3")
    if not exe:
        return {"status": "rocprofv3 not found"}
    out = {}
    per = {}   # kernel -> counter -> [values per dispatch]
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="smx_pmc_", dir="/tmp")
        cmd = [exe, "--pmc", counter, "--kernel-include-regex", "k_", "-d", d, "-o", "p",
               "--output-format", "csv", "--", sys.executable, os.path.join(REPO, "bench.py"),
               "--steps", "2", "--warmup", "1", "--config", args.config, "--no-cpu-baseline",
               "--no-pmc", "--no-e2e", "--no-async", "--no-breakdown"]
        if args.n_ops:
            cmd += ["--n-ops", str(args.n_ops)]
        if args.n_sym:
            cmd += ["--n-sym", str(args.n_sym)]
        env = dict(os.environ, TMPDIR="/tmp")
        try:
            r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL,
                               stderr=subprocess.PIPE, timeout=240)
        except subprocess.TimeoutExpired:
            return {"status": f"{counter} pass timed out"}
        if r.returncode != 0:
            return {"status": f"{counter} pass failed rc={r.returncode}: "
                              + r.stderr.decode(errors="replace")[-200:]}
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        for f in files:
            for row in csv.DictReader(open(f)):
                name = row["Kernel_Name"].split("(")[0].replace("void ", "").strip()
                per.setdefault(name, {}).setdefault(row["Counter_Name"], []).append(
                    float(row["Counter_Value"]))
        shutil.rmtree(d, ignore_errors=True)
    merges = 3  # warm-up + 2 timed steps in the child

    def kbytes(vals, factor):
        return sum(vals) * 1024.0 * factor

    tot = 0.0
    kern = {}
    for k, cs in per.items():
        b = (kbytes(cs.get("FETCH_SIZE", []), FETCH_FACTOR)
             + kbytes(cs.get("WRITE_SIZE", []), WRITE_FACTOR)) / merges
        kern[k] = round(b)
        tot += b
    out["pipeline_traffic"] = round(tot)
    out["per_kernel"] = dict(sorted(kern.items(), key=lambda x: -x[1])[:12])   # bytes per merge
    out["per_kernel_all"] = {k.replace(" ", ""): v for k, v in kern.items()}
    out["factors"] = {"FETCH_SIZE": FETCH_FACTOR, "WRITE_SIZE": WRITE_FACTOR,
                      "note": "FETCH_SIZE x2 is calibrated on streaming reads (DESIGN.md §5); for "
                              "gather-dominated kernels (k_emit4) the x2 figure is an upper bound "
                              "and x1 the lower bound"}
    out["status"] = "ok"
    return out


def cpu_baseline(soa, args) -> dict:
    from concurrent.futures import ThreadPoolExecutor

    from oracle import compose_ref, oracle  # test infrastructure: the checker, timed here
    from semantic_merge_amd.marshal import SoA

    def sample(half):
        half = min(half, soa.n_a, soa.n_b)
        idx = np.concatenate([np.arange(half), soa.n_a + np.arange(half)])
        return SoA(half, half, soa.kind[idx], soa.ts[idx], soa.oid_hi[idx], soa.oid_lo[idx],
                   soa.sym[idx], soa.v0[idx], soa.v1[idx], soa.n_sym)

    s1 = sample(args.cpu_sample // 2)
    t0 = time.perf_counter()
    oracle.compose(s1)
    dt = time.perf_counter() - t0
    res = {"value": round(s1.n / dt, 1), "unit": "ops/s", "cores": 1, "kind": "port",
           "host_cpu_count": os.cpu_count(),
           "sample": f"first {s1.n_a:,} ops of each branch of the same workload ({s1.n:,} ops) "
                     f"through oracle/compose_ref.c, 1 thread, {dt:.1f}s"}
    legs = {}
    # every host thread this job may use at once: independent merges (ctypes releases
    # the GIL).  On the GPU box os.cpu_count() reports the whole machine while the job's
    # CPU share is OMP_NUM_THREADS (16); both are reported.
    host_cpus = os.cpu_count() or 1
    threads = max(1, min(host_cpus, int(os.environ.get("OMP_NUM_THREADS") or host_cpus)))
    sN = sample(args.cpu_sample // 8)
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda _: oracle.compose(sN), range(threads)))
    dtN = time.perf_counter() - t0
    legs["c_port_all_threads"] = {"value": round(threads * sN.n / dtN, 1), "cores": threads,
                                  "host_cpu_count": host_cpus,
                                  "sample": f"{threads} independent {sN.n:,}-op merges, {dtN:.1f}s"}
    sp = sample(200_000)
    t0 = time.perf_counter()
    compose_ref.compose(sp)
    dtp = time.perf_counter() - t0
    legs["python_restatement_1core"] = {"value": round(sp.n / dtp, 1), "cores": 1,
                                        "sample": f"{sp.n:,} ops through oracle/compose_ref.py, {dtp:.1f}s"}
    legs["reference_python_build_container"] = {
        "value": REF_PY_OPS_S, "cores": 1,
        "sample": "reference semmerge compose_oplogs on 1M config-2 ops, measured in the build "
                  "container (Xeon), not on this host (SURVEY.md §3.4, BASELINE.md)"}
    res["legs"] = legs
    return res


def end_to_end(n_ops: int) -> dict:
    """The drop-in compose_oplogs on Op objects (config-2 shape), split into its legs."""
    from semantic_merge_amd import synth
    from semantic_merge_amd._lib import compose_soa, session
    from semantic_merge_amd.marshal import marshal_native
    from semantic_merge_amd.materialize import materialize_conflicts, materialize_ops_native
    from semantic_merge_amd.oplog import ops_from_dicts

    logs = synth.lift_logs(synth.LiftSpec(n_ops, max(n_ops // 100, 1), 7))
    A, B = synth.lift_op_dicts(logs)
    oa, ob = ops_from_dicts(A), ops_from_dicts(B)
    compose_soa(marshal_native(oa[:100], ob[:100]))  # warm the device path
    t = [time.perf_counter()]
    soa = marshal_native(oa, ob)
    t.append(time.perf_counter())
    order, addr, file, ctx, pairs = session().compose(soa, copy=False)  # (as compose_oplogs)
    t.append(time.perf_counter())
    ops = oa + ob
    out = materialize_ops_native(ops, soa.kind, soa.strings, order, addr, file, ctx)
    materialize_conflicts(ops, pairs)
    t.append(time.perf_counter())
    tot = t[3] - t[0]
    return {"n_ops": n_ops, "composed": len(out), "ops_per_s": round(n_ops / tot, 1),
            "marshal_s": round(t[1] - t[0], 4), "device_s": round(t[2] - t[1], 4),
            "materialize_s": round(t[3] - t[2], 4), "total_s": round(tot, 4),
            "note": "compose_oplogs drop-in on Op objects; device_s includes host<->device copies"}


def small_merge(n_ops: int = 1000, reps: int = 50) -> dict:
    """A CLI-sized merge (one diff per branch): the device leg on resident buffers
    (DeviceCompose.run + its sync; the one-workgroup plan) and the whole drop-in on Op
    objects (marshal, device with its copies, materialise); medians."""
    import torch
    from semantic_merge_amd import synth
    from semantic_merge_amd._lib import DeviceCompose, session
    from semantic_merge_amd.marshal import marshal_native
    from semantic_merge_amd.materialize import materialize_conflicts, materialize_ops_native
    from semantic_merge_amd.oplog import ops_from_dicts

    logs = synth.lift_logs(synth.LiftSpec(n_ops, max(n_ops // 100, 10), 7))
    soa = synth.lift_soa(logs)
    dc = DeviceCompose(soa)
    for _ in range(5):
        dc.run()
    torch.cuda.synchronize()
    td = []
    for _ in range(reps):
        t0 = time.perf_counter()
        dc.run()
        torch.cuda.synchronize()
        td.append(time.perf_counter() - t0)
    plan = DeviceCompose.last_plan()
    A, B = synth.lift_op_dicts(logs)
    oa, ob = ops_from_dicts(A), ops_from_dicts(B)
    ops = oa + ob
    te, legs = [], []
    sess = session()  # (the drop-in's: _lib.dropin_session holds it the same way)
    for _ in range(max(reps // 2, 1)):
        t0 = time.perf_counter()
        sa = marshal_native(oa, ob, sess.staging(len(oa) + len(ob)))  # (as compose_oplogs)
        t1 = time.perf_counter()
        order, addr, file, ctx, pairs = sess.compose(sa, copy=False)
        t2 = time.perf_counter()
        materialize_ops_native(ops, sa.kind, sa.strings, order, addr, file, ctx)
        t3 = time.perf_counter()
        materialize_conflicts(ops, pairs)
        t4 = time.perf_counter()
        te.append(t4 - t0)
        legs.append((t1 - t0, t2 - t1, t3 - t2, t4 - t3))
    lm = np.median(np.array(legs), axis=0) * 1e3
    return {"n_ops": n_ops, "plan": plan, "device_ms": round(float(np.median(td)) * 1e3, 4),
            "dropin_ms": round(float(np.median(te)) * 1e3, 4),
            "dropin_legs_ms": {"marshal": round(float(lm[0]), 4), "compose_soa": round(float(lm[1]), 4),
                               "materialize": round(float(lm[2]), 4), "conflicts": round(float(lm[3]), 4),
                               "conflicts_n": int(len(pairs))},
            "note": "device_ms: smx_compose on resident buffers + one sync; dropin_ms: compose_oplogs "
                    "on Op objects (marshal, copies, device, materialise); dropin_legs_ms: medians of "
                    "each leg"}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--n-ops", type=int, default=0, help="override the config's op count")
    ap.add_argument("--n-sym", type=int, default=0, help="override the config's symbol count")
    ap.add_argument("--cpu-sample", type=int, default=40_000_000,
                    help="ops in the 1-thread CPU-baseline sample (rank 0, N=1 only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 traffic passes")
    ap.add_argument("--no-e2e", action="store_true", help="skip the drop-in end-to-end leg")
    ap.add_argument("--no-async", action="store_true", help="skip the smx_compose_async pipeline leg")
    ap.add_argument("--no-breakdown", action="store_true",
                    help="skip the untimed per-stage breakdown leg (the PMC child: exactly 3 merges)")
    ap.add_argument("--e2e-ops", type=int, default=100_000)
    ap.add_argument("--verify", action="store_true", help="check GPU == oracle (slow, N = 1)")
    ap.add_argument("--weak", action="store_true", help="N > 1: N x the config's ops (weak scaling)")
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
    strong = sharded and not args.weak
    n_job = spec.n_total if strong else world * spec.n_total   # ops of the whole job per step
    t0 = time.time()
    sc = dc = None
    if sharded:
        from semantic_merge_amd import shard
        rank_spec = synth.LiftSpec(**{**spec.__dict__, "n_total": spec.n_total // world}) if strong else spec
        soa, na_g, nb_g = synth.lift_slice_soa(rank_spec, rank, world)
        sl_a, sl_b, _, _ = shard.slices_from_soa(soa, 0, 1, dev)
        sl_a.start = sl_b.start = rank * soa.n_a          # this rank's index slice of each branch
        log(f"[rank {rank}] generated slice of {soa.n:,} ops in {time.time() - t0:.1f}s")
        sc = shard.ShardedCompose(sl_a, sl_b, na_g, nb_g, soa.n_sym, shard.Comm(), dev, mode="range")
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

    # a stream of its own (not the null stream)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    lib = _lib.lib()
    # the timed steps carry HIP events around the roofline kernels' stages only (an event
    # pair around every stage of every merge cost ~2% of config 3's step), and only in the
    # last ROOF_STEPS of them.  The full per-stage breakdown comes from an untimed leg
    # after them.
    names = [lib.smx_stage_name(i).decode() for i in range(32)]
    lib.smx_set_profiling_stages(sum(1 << i for i, nm in enumerate(names) if nm in ROOF_STAGES))
    lib.smx_set_profiling(1)
    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize(dev)
    lib.smx_reset_stage_times()
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    # the roofline kernel's launches are timed (HIP events) in the last ROOF_STEPS steps of
    # the timed region (steady state); the others run without events (each event pair
    # drains the queue around the kernel: ~18 us per config-3 merge)
    roof_from = args.steps - min(args.steps, ROOF_STEPS)
    lib.smx_set_profiling(0)
    t0 = time.perf_counter()
    for i in range(args.steps):
        if i == roof_from:
            lib.smx_set_profiling(1)
        run()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    lib.smx_set_profiling(0)
    plan = _lib.DeviceCompose.last_plan()
    stages = _lib.stage_times()
    # per-stage breakdown (every stage timed), outside the timed region
    lib.smx_set_profiling_stages(0xFFFFFFFF)
    stages_all, n_breakdown = stages, args.steps
    if not args.no_breakdown:
        lib.smx_reset_stage_times()
        lib.smx_set_profiling(1)
        n_breakdown = min(args.steps, 5)
        for _ in range(n_breakdown):
            run()
        torch.cuda.synchronize(dev)
        lib.smx_set_profiling(0)
        stages_all = _lib.stage_times()
        lib.smx_reset_stage_times()
    if sharded:
        k, nconf = sc.totals()
    else:
        k, nconf = (int(x) for x in dc.counts.cpu().tolist())
    elapsed = max_over_ranks(elapsed, dev)

    # The same merges through smx_compose_async, all enqueued back to back and one
    # smx_compose_finish after the last: what a caller pipelining merges gets (no host
    # sync between merges).  Reported beside the headline, outside its timed region.
    async_api = None
    if not sharded and world == 1 and not args.no_async and plan != "presorted":
        # only the presorted plan completes inside smx_compose_async: any other plan
        # returns -2 there and runs in smx_compose_finish, one merge per finish
        async_api = {"status": f"plan {plan}: each merge needs its own smx_compose_finish (not pipelined)"}
    elif not sharded and world == 1 and not args.no_async:
        for _ in range(2):  # (the merge's key is seen, then captured as a graph, untimed)
            dc.run_async()
        dc.finish()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for _ in range(args.steps):
            dc.run_async()
        dc.finish()
        torch.cuda.synchronize(dev)
        el_async = time.perf_counter() - t1
        k2, _ = (int(x) for x in dc.counts.cpu().tolist())
        if k2 == k and _lib.DeviceCompose.last_plan() == "presorted":  # every enqueued merge was complete
            async_api = {"ms_per_step": round(el_async / args.steps * 1e3, 4),
                         "value": round(n_job * args.steps / el_async, 1),
                         "note": "smx_compose_async per merge, one smx_compose_finish after the last"}
        else:
            async_api = {"status": "plan needed the synchronous fallback"}

    # The same merges with the timers off (what a caller gets: direct launches).
    graph_api = None
    if not sharded and world == 1 and not args.no_async:
        for _ in range(2):
            run()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for _ in range(args.steps):
            run()
        torch.cuda.synchronize(dev)
        el_graph = time.perf_counter() - t1
        graph_api = {"ms_per_step": round(el_graph / args.steps * 1e3, 4),
                     "value": round(n_job * args.steps / el_graph, 1),
                     "note": "smx_compose per merge, stage timers off"}

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
    value = job_throughput(n_job, 1, args.steps, elapsed)
    # the dominant kernel of the plan that ran: the largest stage time per merge
    roof_stage = max(ROOF_STAGES, key=lambda k: stages.get(k, (0.0, 0))[0])
    roof_kernel, roof_bpo = ROOF_STAGES[roof_stage]
    st_ms, st_calls = stages.get(roof_stage, (0.0, 0))
    # per launch of the kernel (one segsort stage call covers both branch launches of a
    # merge, and its 52 B/op both branches' bytes)
    win_avg = st_ms / max(st_calls, 1)
    achieved = roof_bpo * n / (win_avg * 1e-3) / 1e9 if win_avg > 0 else None
    pipe_gbs = (PIPE_BYTES_PER_OP * n_job + 8 * nconf) / (ms_step * 1e-3) / 1e9

    solo = world == 1
    pmc = pmc_traffic(args) if solo and not args.no_pmc else None
    cpu = cpu_baseline(soa, args) if solo and not args.no_cpu_baseline else None
    e2e = None
    small = None
    if solo and not args.no_e2e:
        try:
            e2e = end_to_end(args.e2e_ops)
        except Exception as exc:  # reported, never fatal for the headline
            e2e = {"status": f"failed: {exc}"}
        try:
            small = small_merge()
        except Exception as exc:
            small = {"status": f"failed: {exc}"}

    if strong:
        par = f"key-range shards x{world}, strong scaling (packed RCCL all-to-all + all-gathers + MAX all-reduce)"
    elif sharded:
        par = f"key-range shards x{world}, weak scaling (packed RCCL all-to-all + all-gathers + MAX all-reduce)"
    else:
        par = f"independent merges x{world}" if world > 1 else "single GPU"
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "ops/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        # N > 1 splits one merge over the ranks by default (strong); N = 1 is that
        # curve's first point.  --weak / --independent keep the per-GPU work fixed.
        "scaling": "weak" if (args.weak or args.independent) else "strong",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (lift-shaped op logs generated from a seed, SURVEY §8(d))",
        "config": {
            "workload": (f"{args.config}: one merge of {n_job:,} ops ({n:,} per GPU), "
                         f"{soa.n_sym:,} symbols, {spec.ops_per_ms} ops/ms, seed {spec.seed}"
                         + (", sharded by timestamp key range" if sharded else "")
                         + (f", {world} independent merges" if world > 1 and not sharded else "")),
            "n_ops_per_gpu": n,
            "n_ops_total": n_job,
            "n_sym": soa.n_sym,
            "composed_ops": k,
            "conflicts": nconf,
            "plan": plan,
            "parallelism": par,
        },
        # SURVEY §8(d)'s quantity: 53 B/op (+8 B per conflict) of the whole merge over the
        # wall time of smx_compose (every kernel of the merge and its one host sync);
        # traffic = the PMC-measured HBM bytes of all of the merge's kernels
        "roofline": {
            "bound": "hbm",
            "kernel": "smx_compose (the whole merge: every kernel, one host sync)",
            "achieved": round(pipe_gbs, 1),
            "peak": HBM_PEAK_GBS * world,
            "unit": "GB/s",
            "frac": round(pipe_gbs / (HBM_PEAK_GBS * world), 4),
            "traffic": pmc.get("pipeline_traffic") if pmc and pmc.get("status") == "ok" else None,
            "bytes_per_op": PIPE_BYTES_PER_OP,
            "ms_per_merge": round(ms_step, 4),
        },
        # the plan's dominant kernel alone: its own algorithmic bytes over its average
        # launch time (HIP events on the call's stream inside the timed region)
        "kernel_roofline": {
            "bound": "hbm",
            "kernel": roof_kernel + (" (both branches)" if roof_stage == "segsort" else ""),
            "achieved": round(achieved, 1) if achieved else None,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
            # HBM bytes per merge of that kernel (PMC passes; per launch for the one-launch
            # kernels, both branch launches for the segmented sort)
            "traffic": round(sum(v for k2, v in pmc.pop("per_kernel_all").items() if k2.startswith(roof_kernel)))
            if pmc and pmc.get("status") == "ok" else None,
            "bytes_per_op": roof_bpo,
            "avg_launch_ms": round(win_avg, 4),
            "timed_launches": int(st_calls),
        },
        "pmc": pmc,
        # per merge: each stage's summed time over its launches in one merge, and how many
        # times the merge entered it (breakdown leg: every stage timed, n_breakdown merges)
        "stages_ms_per_step": {k2: round(v[0] / n_breakdown, 4) for k2, v in stages_all.items() if v[1]},
        "stage_calls_per_step": {k2: round(v[1] / n_breakdown, 2) for k2, v in stages_all.items() if v[1]},
        "cpu_baseline": cpu,
        "end_to_end": e2e,
        "small_merge": small,
        "async_api": async_api,
        "graph_api": graph_api,
    }
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
