"""GPU parity of the sharded single merge (semantic_merge_amd/shard.py): 2-3 ranks on one
GPU over gloo (collectives through host copies; RCCL runs the same code on a node).
Each rank starts from an index slice of the global logs; the assembled per-shard outputs
must equal the CPU oracle's composition of the whole merge, bit for bit."""
import os
import queue
import shutil
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _init(rank, world, store_path, backend="gloo"):
    """Process group over a FileStore: no port to race for (a bound-then-freed port
    handed to the children can be taken before rank 0 listens on it), and no eager
    communicator set-up for RCCL (it is created by the first collective)."""
    import torch
    import torch.distributed as dist
    store = dist.FileStore(store_path, world)
    if backend == "nccl":  # RCCL: one rank per GPU
        torch.cuda.set_device(0)
    dist.init_process_group(backend, store=store, rank=rank, world_size=world)


def _phase(q, rank, name):
    q.put(("phase", rank, name))


def _spawn(target, world, extra, timeout):
    """Start `world` ranks of target(rank, world, store_path, q, *extra) and collect one
    ("done", rank, payload) per rank.  Ranks report ("phase", rank, name) as they go;
    if nothing arrives for `timeout` seconds the ranks are killed and the failure names
    each rank's last phase."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    tmp = tempfile.mkdtemp(prefix="smx_store_")
    store_path = os.path.join(tmp, "store")
    procs = [ctx.Process(target=target, args=(r, world, store_path, q) + tuple(extra)) for r in range(world)]
    for p in procs:
        p.start()
    got, last = {}, {r: "spawned" for r in range(world)}
    try:
        while len(got) < world:
            try:
                msg = q.get(timeout=timeout)
            except queue.Empty:
                raise AssertionError(f"no progress for {timeout} s; last phase per rank: {last}") from None
            if msg[0] == "phase":
                last[msg[1]] = msg[2]
            else:
                got[msg[1]] = msg[2]
        for p in procs:
            p.join(60)
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(10)
        shutil.rmtree(tmp, ignore_errors=True)
    return got


def _make(case):
    from semantic_merge_amd import synth
    kind, n, n_sym, seed = case
    if kind == "chain":
        return _chain_soa(n, seed)
    if kind == "c2s":  # config 2's shape, shuffled branch logs (any order)
        spec = synth.LiftSpec(**{**synth.CONFIGS["c2s"].__dict__, "n_total": n, "n_sym": n_sym,
                                 "seed": seed})
        return synth.lift_soa(synth.lift_logs(spec))
    if kind == "hollow":  # 4 ranks: a run of equal timestamps makes shard 1 empty
        return _hollow_soa(n, seed)
    if kind == "dense":  # long equal-timestamp groups: windows overflow, ORDER_FIX repairs
        spec = synth.LiftSpec(n, n_sym, seed, ops_per_ms=4096)
        return synth.lift_soa(synth.lift_logs(spec))
    if kind == "dense_unordered":  # ... and two ops of A's first quarter swapped across ms groups
        soa = _make(("dense", n, n_sym, seed))
        i, j = 100, soa.n_a // 4
        assert soa.ts[i] < soa.ts[j]
        for f in ("kind", "ts", "oid_hi", "oid_lo", "sym", "v0", "v1"):
            a = getattr(soa, f)
            a[i], a[j] = a[j].copy(), a[i].copy()
        return soa
    if kind == "wide_value":  # one move's address id too wide for the 32-bit partial tables
        soa = _make(("lift", n, n_sym, seed))
        mv = np.flatnonzero(soa.kind == 0)
        # every move of one symbol: its shard's last writer of the address is then wide
        s = soa.sym[mv[len(mv) // 3]]
        soa.v0[mv[soa.sym[mv] == s]] = (1 << 30) + 7
        return soa
    if kind == "lift":
        spec = synth.LiftSpec(n, n_sym, seed, ops_per_ms=64)
    elif kind == "adv":  # rename-heavy, 30% of symbols renamed on both sides: many conflicts
        spec = synth.LiftSpec(n, n_sym, seed, ops_per_ms=256, mix=synth.ADVERSARIAL_MIX,
                              rename_overlap=0.30, divergent=0.2)
    else:
        raise ValueError(kind)
    soa = synth.lift_soa(synth.lift_logs(spec))
    if kind == "lift" and seed % 2 == 1:
        # moves with a None newAddress / newFile: the prefix fix-up crosses shards
        rng = np.random.default_rng(seed)
        mv = np.flatnonzero(soa.kind == 0)
        soa.v0[mv[rng.random(len(mv)) < 0.3]] = -1
        soa.v1[mv[rng.random(len(mv)) < 0.2]] = -1
    return soa


def _chain_soa(n_ren, seed):
    """One long DivergentRename region: branch A renames symbol 0 n_ren times before
    any of branch B's n_ren renames of it (other names), plus edits.  Every A rename
    conflicts with the B rename d ahead, so d climbs to n_ren and the region spans
    both shards: it is open at shard 0's end and handed to shard 1."""
    from semantic_merge_amd.marshal import SoA
    rng = np.random.default_rng(seed)
    n_edit = n_ren // 2
    na = nb = n_ren + n_edit
    kind = np.full(na + nb, 10, np.uint8)            # editStmtBlock precedence rank
    kind[:n_ren] = 1
    kind[na:na + n_ren] = 1
    ts = np.concatenate([np.arange(na, dtype=np.uint64) * 2,
                         np.uint64(10 * na) + np.arange(nb, dtype=np.uint64) * 2])
    hi = rng.integers(0, 2**63, size=na + nb, dtype=np.int64).astype(np.uint64)
    lo = rng.integers(0, 2**63, size=na + nb, dtype=np.int64).astype(np.uint64)
    sym = np.zeros(na + nb, np.uint32)
    sym[n_ren:na] = rng.integers(1, 5, size=n_edit)
    sym[na + n_ren:] = rng.integers(1, 5, size=n_edit)
    v0 = np.full(na + nb, -1, np.int32)
    v1 = np.full(na + nb, -1, np.int32)
    v0[:n_ren], v1[:n_ren] = 0, 0
    v0[na:na + n_ren], v1[na:na + n_ren] = 1, 1
    return SoA(na, nb, kind, ts, hi, lo, sym, v0, v1, 5, ["a", "b"])


def _hollow_soa(n_ren, seed):
    """A renames symbol 0 n_ren times (name class 0), B n_ren times (class 1) after all
    of A: one DivergentRename region from shard 0 to the last shard.  A's ops
    n_ren/4 .. n_ren/2 share one timestamp, so with 4 ranks the splitters of shards 1 and
    2 coincide and shard 1 is empty: the open region must pass through it, and what it
    hands on changes between walk rounds."""
    from semantic_merge_amd.marshal import SoA
    rng = np.random.default_rng(seed)
    na = nb = n_ren
    ts_a = np.arange(na, dtype=np.uint64) * 2
    q1, q2 = na // 4, na // 2
    ts_a[q1:q2 + 1] = ts_a[q1]
    ts = np.concatenate([ts_a, np.uint64(10 * na) + np.arange(nb, dtype=np.uint64) * 2])
    hi = rng.integers(0, 2**63, size=na + nb, dtype=np.int64).astype(np.uint64)
    lo = rng.integers(0, 2**63, size=na + nb, dtype=np.int64).astype(np.uint64)
    kind = np.full(na + nb, 1, np.uint8)
    sym = np.zeros(na + nb, np.uint32)
    v0 = np.concatenate([np.zeros(na, np.int32), np.ones(nb, np.int32)])
    return SoA(na, nb, kind, ts, hi, lo, sym, v0, v0.copy(), 1, ["a", "b"])


def _worker(rank, world, store_path, q, case, halo, mode="auto", backend="gloo"):
    import torch.distributed as dist
    _phase(q, rank, "init_process_group")
    _init(rank, world, store_path, backend)
    try:
        from semantic_merge_amd import shard
        _phase(q, rank, "make inputs")
        soa = _make(case)
        a, b, na, nb = shard.slices_from_soa(soa, rank, world, "cuda:0")
        _phase(q, rank, "ShardedCompose")
        sc = shard.ShardedCompose(a, b, na, nb, soa.n_sym, shard.Comm(), "cuda:0", halo_cap=halo,
                                  mode=mode)
        _phase(q, rank, "run 1")
        sc.run()
        res = sc.results()
        first = (res, sc.totals())
        _phase(q, rank, "run 2")
        sc.run()  # a second run on the same buffers (bench.py's steps) gives the same results
        res2 = sc.results()
        same = all(np.array_equal(x, y) for x, y in zip(first[0][:5], res2[:5]))
        _phase(q, rank, "destroy_process_group")
        q.put(("done", rank, (res, sc.in_state, (sc.exchange_mode, same, first[1], sc.order_fixes,
                                                 sc.tab32_used, sc.tab_redo))))
    except Exception as e:  # report to the parent instead of hanging the collective
        q.put(("done", rank, (repr(e), None, None)))
        raise
    finally:
        dist.destroy_process_group()


def _run(case, world, halo=4096, mode="auto", backend="gloo"):
    got = _spawn(_worker, world, (case, halo, mode, backend), timeout=180)
    for r in range(world):
        assert not isinstance(got[r][0], str), f"rank {r}: {got[r][0]}"
    return [got[r][0] for r in range(world)], got


def _check(case, world, halo=4096, mode="auto", want_mode=None, backend="gloo"):
    from oracle import oracle
    from semantic_merge_amd import shard
    parts, got = _run(case, world, halo, mode, backend)
    glob = shard.assemble(parts)
    ref = oracle.compose(_make(case))
    names = ("order", "addr", "file", "ctx", "conflicts")
    for name, g, r in zip(names, glob, ref):
        assert g.shape == r.shape, f"{case} x{world}: {name} shape {g.shape} vs {r.shape}"
        assert np.array_equal(g, r), f"{case} x{world}: {name} differs"
    for r in range(world):
        emode, same, totals = got[r][2][:3]
        assert same, f"rank {r}: a second run differs"
        assert totals == (len(ref[0]), len(ref[4])), totals
        if want_mode:
            assert emode == want_mode, emode
    return got, ref


@pytest.mark.parametrize("mode", ["range", "sample"])
def test_shard_rccl_single_rank(mode):
    """The RCCL branch of shard.Comm (collectives on device tensors: all_gather_into_tensor,
    MAX all_reduce on int64, all_to_all_single of packed uint8 records) on one GPU: a
    one-rank "nccl" group runs the whole sharded step sequence, checked against the oracle.
    (More ranks need one GPU each: the driver's node.)"""
    _check(("lift", 60_000, 2_000, 5), 1, mode=mode, backend="nccl",
           want_mode=None)


def test_shard_lift_two_ranks():
    _check(("lift", 200_000, 2_000, 4), 2)


def test_shard_lift_none_moves_three_ranks():
    _check(("lift", 150_000, 1_000, 5), 3)


def test_shard_adversarial_conflicts_cross_boundaries():
    # 8 symbols: natural heads collide constantly, regions are long and cross shards
    got, ref = _check(("adv", 120_000, 8, 8), 3)
    assert len(ref[4]) > 1000  # conflict-dense
    handed = [got[r][1] for r in range(3) if got[r][1] != (0, 0)]
    print("incoming open regions:", handed)


def test_shard_open_region_handed_to_next_shard():
    got, ref = _check(("chain", 3000, 0, 3), 2)
    assert len(ref[4]) == 3000
    assert got[1][1] != (0, 0), "shard 1 must receive the open region"


def test_shard_halo_too_short_fails_loudly():
    with pytest.raises(AssertionError, match="halo"):
        _check(("chain", 3000, 0, 3), 2, halo=16)


def test_shard_tiny_with_empty_shards():
    _check(("lift", 40, 5, 2), 3)


def test_shard_open_region_through_empty_middle_shard():
    got, ref = _check(("hollow", 4000, 0, 5), 4)
    assert len(ref[4]) == 4000
    assert got[1][0][0].size == 0, "shard 1 must be empty"
    assert got[2][1] != (0, 0) and got[3][1] != (0, 0), "the region must reach shards 2 and 3"


def test_shard_sample_sort_shuffled_c2s():
    """Branch logs in any order (config 2s's shape): the sample-sort exchange on the full
    T key, the generic plan per shard, global sources through src_map."""
    _check(("c2s", 300_000, 3_000, 7), 3, want_mode="sample")


def test_shard_sample_sort_forced_on_ordered_logs():
    _check(("adv", 80_000, 16, 3), 2, mode="sample", want_mode="sample")


def test_shard_dense_ties_order_fix():
    # 4096 ops per timestamp: presorted windows overflow on the first (asynchronous)
    # ORDER; ORDER_FIX retries with smaller windows
    got, _ = _check(("dense", 200_000, 2_000, 6), 2, want_mode="range")
    assert any(got[r][2][3] for r in range(2)), "ORDER_FIX did not run"


def test_shard_eight_ranks_range_config2_shape():
    """The 8-GPU node's geometry on one GPU (8 gloo ranks): 7 splitters, halos and open
    regions across 7 boundaries, an 8-way MAX all-reduce; config 2's shape (1M ops, 10k
    symbols) with None-valued moves whose prefix crosses shards, timestamp ranges."""
    _check(("lift", 1_000_000, 10_000, 7), 8, want_mode="range")


def test_shard_eight_ranks_32bit_tables():
    """Eight ranks without None-valued moves: the speculative tables go through the
    32-bit all-reduce (rank tag in the top 4 bits) and are final -- no 64-bit redo."""
    got, _ = _check(("lift", 800_000, 10_000, 8), 8, want_mode="range")
    assert all(got[r][2][4] == 2 for r in range(8)), [got[r][2][4] for r in range(8)]  # (two runs)


def test_shard_32bit_table_overflow_redone_wide():
    """A value too wide for the 32-bit partial tables (2 ranks: 2 tag bits, 29 value bits)
    sets the shard's overflow flag (PartTab::put), the speculative tables are discarded and
    every rank redoes them with 64-bit entries -- same output as the single merge."""
    got, _ = _check(("wide_value", 200_000, 2_000, 4), 2, want_mode="range")
    assert all(got[r][2][4] == 2 for r in range(2))   # the speculative 32-bit step ran (two runs)
    assert all(got[r][2][5] == 2 for r in range(2)), [got[r][2][5] for r in range(2)]  # ... and was redone


def test_shard_eight_ranks_sample_sort_shuffled():
    _check(("c2s", 400_000, 4_000, 7), 8, want_mode="sample")


def test_shard_eight_ranks_open_region_across_shards():
    """One DivergentRename region from the first shard holding B's renames to the last:
    it is open at several shard ends and handed on, shard by shard."""
    got, ref = _check(("chain", 3000, 0, 3), 8)  # (depth <= 3000: inside the 4096-rename halo)
    assert len(ref[4]) == 3000
    handed = [r for r in range(8) if got[r][1] != (0, 0)]
    assert len(handed) >= 2, handed


def test_shard_range_unordered_dense_slice_fails_loudly():
    """mode "range" trusts the ORDER step to reject a slice whose timestamps decrease.
    With dense ties the presorted plan's early verdict (a group no window holds) hides the
    window kernel's order check, so ORDER_FIX runs the segmented sort, which reports the
    decrease itself: the step must fail on every rank, never radix-sort the slice locally
    (that orders it within the shard but not across the shards)."""
    with pytest.raises(AssertionError, match="timestamp-ordered"):
        _check(("dense_unordered", 200_000, 2_000, 6), 2, mode="range")


def test_shard_tables_twice_without_scatter_rejected():
    """SMX_SHARD_TABLES consumes the bucketed records (the walk's skips are applied in
    place): a second TABLES without SCATTER in between is an argument error."""
    import ctypes as C
    import torch
    import torch.distributed as dist
    from semantic_merge_amd import _abi, _lib, shard, synth
    store = tempfile.mkdtemp(prefix="smx_store_")
    dist.init_process_group("gloo", store=dist.FileStore(os.path.join(store, "s"), 1), rank=0, world_size=1)
    try:
        soa = synth.lift_soa(synth.lift_logs(synth.LiftSpec(20_000, 200, 3)))
        a, b, na, nb = shard.slices_from_soa(soa, 0, 1, "cuda:0")
        sc = shard.ShardedCompose(a, b, na, nb, soa.n_sym, shard.Comm(), "cuda:0", mode="range")
        sc.run()
        sc._step(_abi.SHARD_SCATTER)
        sc._step(_abi.SHARD_TABLES)
        with pytest.raises(_lib.SmxError, match="TABLES"):
            sc._step(_abi.SHARD_TABLES)
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
        shutil.rmtree(store, ignore_errors=True)


def test_bench_two_ranks_sharded():
    """bench.py's N > 1 path (one sharded merge, torchrun) end to end, 2 ranks on this
    GPU over gloo: one JSON line with the whole-job rate; strong scaling by default
    (the config's ops split over the ranks), weak with --weak."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SMX_BENCH_BACKEND="gloo")
    for extra, total, scaling in (([], 2_000_000, "strong"), (["--weak"], 4_000_000, "weak")):
        # --standalone: the launcher binds its own rendezvous store on an OS-chosen port
        # (no port picked here and handed over, which another process could take first)
        cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
               "--nproc-per-node", "2", "bench.py",
               "--gpus", "2", "--steps", "2", "--warmup", "1", "--n-ops", "2000000", "--n-sym",
               "20000"] + extra
        r = subprocess.run(cmd, cwd=repo, env=env, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
        out = json.loads(line)
        assert out["n_gpus"] == 2 and out["config"]["n_ops_total"] == total
        assert out["scaling"] == scaling
        assert out["value"] > 0 and "key-range shards" in out["config"]["parallelism"]


_FIELDS = ("kind", "ts", "oid_hi", "oid_lo", "sym", "v0", "v1")


def _full_worker(rank, world, store_path, q, datadir):
    """One rank of the full-size config-3 merge: its index slices of the global logs,
    memory-mapped from the files the parent wrote (the logs are generated once), one
    sharded run, and this shard's results written back for the parent to assemble."""
    import torch
    import torch.distributed as dist
    _phase(q, rank, "init_process_group")
    _init(rank, world, store_path)
    try:
        _phase(q, rank, "map c3")
        from semantic_merge_amd import shard
        from semantic_merge_amd.marshal import SoA
        meta = np.load(os.path.join(datadir, "meta.npy"))
        cols = {f: np.load(os.path.join(datadir, f + ".npy"), mmap_mode="r") for f in _FIELDS}
        soa = SoA(int(meta[0]), int(meta[1]), n_sym=int(meta[2]), **cols)
        a, b, na, nb = shard.slices_from_soa(soa, rank, world, "cuda:0")
        del soa, cols
        sc = shard.ShardedCompose(a, b, na, nb, int(meta[2]), shard.Comm(), "cuda:0", mode="range")
        del a, b
        _phase(q, rank, "run")
        sc.run()
        res = sc.results()
        _phase(q, rank, "write results")
        np.savez(os.path.join(datadir, f"res_{rank}.npz"), *res[:5], seg=np.asarray(res[5], np.int64))
        del sc
        torch.cuda.empty_cache()
        q.put(("done", rank, None))
    except Exception as e:  # report to the parent instead of hanging the collective
        q.put(("done", rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _full_c3_sharded(world):
    """Config 3 at full size (100M ops, 1M symbols) as ONE merge over `world` key-range
    shards on this GPU (gloo): the assembled output's sha256 against the C oracle's
    digest of the single merge (tests/golden/full_digests.json)."""
    import hashlib
    import json
    from semantic_merge_amd import shard, synth
    rec = {r["name"]: r for r in json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                                             "full_digests.json")))}["c3"]
    base = "/dev/shm" if os.path.isdir("/dev/shm") else None
    datadir = tempfile.mkdtemp(prefix="smx_c3_", dir=base)
    try:
        soa = synth.lift_soa(synth.lift_logs(synth.CONFIGS["c3"]))
        for f in _FIELDS:
            np.save(os.path.join(datadir, f + ".npy"), getattr(soa, f))
        np.save(os.path.join(datadir, "meta.npy"), np.array([soa.n_a, soa.n_b, soa.n_sym], np.int64))
        del soa
        got = _spawn(_full_worker, world, (datadir,), timeout=400)
        for r in range(world):
            assert got[r] is None, f"rank {r}: {got[r]}"
        parts = []
        for r in range(world):
            z = np.load(os.path.join(datadir, f"res_{r}.npz"))
            parts.append(tuple(z[f"arr_{i}"] for i in range(5)) + ([tuple(x) for x in z["seg"].tolist()],))
        glob = shard.assemble(parts)
        h = hashlib.sha256()
        for arr in glob:
            h.update(np.ascontiguousarray(arr, dtype=np.int32).tobytes())
        assert (len(glob[0]), len(glob[4])) == (rec["n_out"], rec["n_conflicts"])
        assert h.hexdigest() == rec["sha256"]
    finally:
        shutil.rmtree(datadir, ignore_errors=True)


@pytest.mark.timeout(900)
def test_shard_full_size_c3_two_ranks():
    _full_c3_sharded(2)


@pytest.mark.timeout(1100)
def test_shard_full_size_c3_eight_ranks():
    """BASELINE config 3's geometry (100M ops over 8 shards) rehearsed on one GPU with
    8 gloo ranks: 7 key-range splitters, halos and region hand-offs at 7 boundaries, an
    8-way MAX all-reduce of 1M-symbol tables -- against the single merge's digest."""
    _full_c3_sharded(8)


@pytest.mark.parametrize("na,nb,offb,order", [(1000, 777, 1200, True), (5, 40, 10, True), (0, 50, 3, True),
                                             (300, 0, 0, True), (300, 200, 400, False)])
def test_range_info_native_matches_reference_layout(na, nb, offb, order):
    """smx_shard_range_info (the range plan's per-rank vector in two launches) against
    the same vector built on the host: sizes, end keys, order flag, signed flags and the
    RH head / tail keys (right-aligned tail, short slices padded with their first key);
    timestamps with the top bit set included."""
    import ctypes as C
    import torch
    from semantic_merge_amd._lib import lib
    from semantic_merge_amd.shard import RH
    rng = np.random.default_rng(na + nb + offb)
    buf = np.zeros(max(5 + na, offb + nb) + 64, dtype=np.uint64)
    a = np.sort(rng.integers(0, 2**64 - 1, na, dtype=np.uint64))
    b = np.sort(rng.integers(0, 2**64 - 1, nb, dtype=np.uint64))
    if not order and nb > 3:
        b[[1, 2]] = b[[2, 1]]  # a decrease inside the B slice
    buf[5:5 + na] = a
    buf[offb:offb + nb] = b
    dev = torch.device("cuda:0")
    t = torch.from_numpy(buf.view(np.int64)).to(dev)
    out = torch.zeros(9 + 4 * RH, dtype=torch.int64, device=dev)
    rc = lib().smx_shard_range_info(t.data_ptr(), 5, na, offb, nb, RH, 1, 1, 0, out.data_ptr(),
                                    torch.cuda.current_stream(dev).cuda_stream)
    assert rc == 0
    got = out.cpu().numpy()

    def key(v):
        return np.int64(np.uint64(v) ^ np.uint64(1 << 63))

    want = [na, nb, key(a[0]) if na else 0, key(a[-1]) if na else 0, key(b[0]) if nb else 0,
            key(b[-1]) if nb else 0, int(bool(np.all(np.diff(a.astype(object)) >= 0)) and
                                         bool(np.all(np.diff(b.astype(object)) >= 0))), 1, 0]
    for x in (a, b):
        n = len(x)
        h = min(RH, n)
        pad = [key(x[0])] if n else [0]
        want += [key(v) for v in x[:h]] + pad * (RH - h)
        want += pad * (RH - h) + [key(v) for v in x[n - h:]]
    assert got.tolist() == [int(w) for w in want]
