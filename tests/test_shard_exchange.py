"""Sharded merge, host side on CPU (gloo, 2-3 ranks): the key-range all-to-all (one
all_to_all_single of packed records) puts every op on the shard owning its timestamp, in
place (headroom), with the global source offsets the kernels need; the originals come
back for the next step.  The sample-sort exchange (logs in any order) puts every op on
the shard owning its full T key, with its global source index.  The compute steps need
a GPU (tests/test_gpu_shard.py)."""
import os
import shutil
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp


def _init(rank, world, store_path):
    # FileStore rendezvous: no bound-then-freed port for the children to race for
    import torch.distributed as dist
    dist.init_process_group("gloo", store=dist.FileStore(store_path, world), rank=rank, world_size=world)


def _store_path():
    return os.path.join(tempfile.mkdtemp(prefix="smx_store_"), "store")


def _soa(n, seed, ops_per_ms, high=False):
    from semantic_merge_amd import synth
    soa = synth.lift_soa(synth.lift_logs(synth.LiftSpec(n, 50, seed, ops_per_ms=ops_per_ms)))
    if high:  # the later half of each branch above 2^63: still ordered as u64, and the
        # ranks holding it take the unsigned splitter search, the others the signed one
        for lo, m in ((0, soa.n_a), (soa.n_a, soa.n_b)):
            soa.ts[lo + m // 2: lo + m] |= np.uint64(1 << 63)
    return soa


def _worker(rank, world, port, args, q):  # port: the FileStore path
    import torch
    import torch.distributed as dist
    _init(rank, world, port)
    try:
        from semantic_merge_amd import shard
        n, seed, opm, headroom, high = args
        soa = _soa(n, seed, opm, high)
        a, b, na, nb = shard.slices_from_soa(soa, rank, world, "cpu")
        sc = shard.ShardedCompose(a, b, na, nb, soa.n_sym, shard.Comm(), "cpu", halo_cap=64,
                                  headroom=headroom)
        sc.exchange()
        assert sc.exchange_mode == "range"
        (a_lo, a_hi), (b_lo, b_hi) = sc.rng
        got = {f: (sc.buf[f][a_lo:a_hi].numpy().copy(), sc.buf[f][b_lo:b_hi].numpy().copy())
               for f in shard.FIELDS}
        sc._restore()
        restored = all(torch.equal(getattr(a, f), sc.buf[f][sc._oa:sc._oa + sc.na_s])
                       and torch.equal(getattr(b, f), sc.buf[f][sc._ob:sc._ob + sc.nb_s])
                       for f in shard.FIELDS)
        q.put((rank, sc.src_a, sc.src_b - na, got, restored, sc.hd))
    except Exception as e:
        q.put((rank, repr(e), None, None, None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,opm,headroom,high", [(2, 20_000, 64, None, False),
                                                       (3, 30_000, 7, None, False),
                                                       (3, 9_000, 1000, 0, False),
                                                       (4, 24_000, 64, None, True),
                                                       # the 8-GPU node's geometry: 7 splitters
                                                       (8, 48_000, 64, None, False),
                                                       (8, 16_000, 333, 0, True)])
def test_exchange_key_ranges(world, n, opm, headroom, high):
    from semantic_merge_amd import shard
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _store_path()
    args = (n, 3, opm, headroom, high)
    procs = [ctx.Process(target=_worker, args=(r, world, port, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        item = q.get(timeout=120)
        res[item[0]] = item
    for p in procs:
        p.join(60)
    shutil.rmtree(os.path.dirname(port), ignore_errors=True)
    errs = [res[r][1] for r in range(world) if isinstance(res[r][1], str)]
    assert not errs, errs
    soa = _soa(n, 3, opm, high)
    na, nb = soa.n_a, soa.n_b
    cols = {"kind": soa.kind, "ts": soa.ts.view(np.int64), "hi": soa.oid_hi.view(np.int64),
            "lo": soa.oid_lo.view(np.int64), "sym": soa.sym.view(np.int32), "v0": soa.v0, "v1": soa.v1}
    ea = eb = 0
    for r in range(world):
        _, sa, sb, got, restored, _ = res[r]
        assert restored
        assert sa == ea and sb == eb          # shards tile each branch in order
        la, lb = len(got["kind"][0]), len(got["kind"][1])
        for f in shard.FIELDS:
            assert np.array_equal(got[f][0], cols[f][sa:sa + la]), (r, f, "A")
            assert np.array_equal(got[f][1], cols[f][na + sb:na + sb + lb]), (r, f, "B")
        ea, eb = sa + la, sb + lb
        # key ranges: every timestamp of shard r is below every timestamp of shard r+1
        if r + 1 < world:
            nxt = res[r + 1][3]
            mine = np.concatenate([got["ts"][0], got["ts"][1]]).view(np.uint64)
            theirs = np.concatenate([nxt["ts"][0], nxt["ts"][1]]).view(np.uint64)
            if len(mine) and len(theirs):
                assert mine.max() < theirs.min()
    assert ea == na and eb == nb
    if headroom == 0:
        assert any(res[r][5] > 0 for r in range(world))  # the headroom grew


def _spawn(target, world, args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _store_path()
    procs = [ctx.Process(target=target, args=(r, world, port, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        item = q.get(timeout=120)
        res[item[0]] = item
    for p in procs:
        p.join(60)
    shutil.rmtree(os.path.dirname(port), ignore_errors=True)
    errs = [res[r][1] for r in range(world) if isinstance(res[r][1], str)]
    assert not errs, errs
    return res


def _shuffled(n, seed, only_a=False):
    from semantic_merge_amd import synth
    if not only_a:
        return synth.lift_soa(synth.lift_logs(synth.LiftSpec(n, 40, seed, ops_per_ms=3, shuffle=True)))
    # branch A in random order, branch B timestamp-ordered (the order flags
    # of the two branches must be combined, not overwritten by B's)
    soa = synth.lift_soa(synth.lift_logs(synth.LiftSpec(n, 40, seed, ops_per_ms=3)))
    perm = np.random.default_rng(seed).permutation(soa.n_a)
    for f in ("kind", "ts", "oid_hi", "oid_lo", "sym", "v0", "v1"):
        col = getattr(soa, f)
        col[:soa.n_a] = col[:soa.n_a][perm]
    return soa


def _sample_worker(rank, world, port, args, q):
    import torch.distributed as dist
    _init(rank, world, port)
    try:
        from semantic_merge_amd import shard
        n, seed, mode, only_a = args
        soa = _shuffled(n, seed, only_a)
        a, b, na, nb = shard.slices_from_soa(soa, rank, world, "cpu")
        sc = shard.ShardedCompose(a, b, na, nb, soa.n_sym, shard.Comm(), "cpu", halo_cap=64,
                                  mode=mode, oversample=32)
        sc.exchange()
        m = sc.n_a + sc.n_b
        got = {f: sc.sbuf[f][:m].numpy().copy() for f in shard.FIELDS}
        q.put((rank, sc.n_a, sc.exchange_mode, got, sc.src_map[:m].numpy().copy()))
    except Exception as e:
        q.put((rank, repr(e), None, None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,mode,only_a", [(2, 6_000, "sample", False), (3, 9_001, "auto", False),
                                                (2, 6_000, "auto", True), (8, 24_000, "sample", False)])
def test_exchange_sample_sort(world, n, mode, only_a):
    """Unordered branch logs: every op lands exactly once on the shard owning its full T
    key (kind, ts, oid, side, index), A' and B' in global index order, shards balanced.
    With mode "auto", one unordered branch is enough to choose the sample sort."""
    from semantic_merge_amd import shard
    res = _spawn(_sample_worker, world, (n, 5, mode, only_a))
    soa = _shuffled(n, 5, only_a)
    cols = {"kind": soa.kind, "ts": soa.ts.view(np.int64), "hi": soa.oid_hi.view(np.int64),
            "lo": soa.oid_lo.view(np.int64), "sym": soa.sym.view(np.int32), "v0": soa.v0, "v1": soa.v1}
    seen = np.zeros(soa.n, np.int64)
    prev_max = None
    for r in range(world):
        _, n_a, emode, got, smap = res[r]
        assert emode == "sample"
        seen[smap] += 1
        for f in shard.FIELDS:
            assert np.array_equal(got[f], cols[f][smap]), (r, f)
        assert np.all(smap[:n_a] < soa.n_a) and np.all(smap[n_a:] >= soa.n_a)
        assert np.all(np.diff(smap[:n_a]) > 0) and np.all(np.diff(smap[n_a:]) > 0)
        assert len(smap) < 2.0 * soa.n / world                       # balanced by the samples
        if len(smap):
            keys = sorted(zip(soa.kind[smap].tolist(), soa.ts[smap].tolist(), soa.oid_hi[smap].tolist(),
                              soa.oid_lo[smap].tolist(), smap.tolist()))
            if prev_max is not None:
                assert prev_max < keys[0]                             # key ranges in shard order
            prev_max = keys[-1]
    assert np.all(seen == 1)


def test_packed_records_round_trip():
    import torch
    from semantic_merge_amd import shard
    rng = np.random.default_rng(1)
    m = 1000
    cols = {"kind": torch.from_numpy(rng.integers(0, 18, m).astype(np.uint8)),
            "ts": torch.from_numpy(rng.integers(-2**62, 2**62, m)),
            "hi": torch.from_numpy(rng.integers(-2**62, 2**62, m)),
            "lo": torch.from_numpy(rng.integers(-2**62, 2**62, m)),
            "sym": torch.from_numpy(rng.integers(0, 2**30, m).astype(np.int32)),
            "v0": torch.from_numpy(rng.integers(-1, 2**30, m).astype(np.int32)),
            "v1": torch.from_numpy(rng.integers(-1, 2**30, m).astype(np.int32))}
    gidx = torch.from_numpy(rng.integers(0, 2**31 - 1, m).astype(np.int32))
    rec = shard.pack_records(cols, gidx)
    assert rec.shape == (m, 41) and rec.dtype == torch.uint8
    assert shard.pack_records(cols).shape == (m, 37)
    back, g = shard.unpack_records(rec, {f: t.dtype for f, t in cols.items()}, with_gidx=True)
    assert all(torch.equal(back[f], cols[f]) for f in cols) and torch.equal(g, gidx)
    empty = shard.pack_records({f: t[:0] for f, t in cols.items()})
    assert empty.shape == (0, 37)


def _strong_worker(rank, world, port, args, q):
    import torch.distributed as dist
    _init(rank, world, port)
    try:
        from semantic_merge_amd import shard, synth
        n_total, = args
        spec = synth.LiftSpec(n_total // world, 300, 9, ops_per_ms=7)    # bench.py's strong split
        soa, na_g, nb_g = synth.lift_slice_soa(spec, rank, world)
        a, b, _, _ = shard.slices_from_soa(soa, 0, 1, "cpu")
        a.start = b.start = rank * soa.n_a
        sc = shard.ShardedCompose(a, b, na_g, nb_g, soa.n_sym, shard.Comm(), "cpu", mode="range")
        sc.exchange()
        (a_lo, a_hi), (b_lo, b_hi) = sc.rng
        ts = np.concatenate([sc.buf["ts"][a_lo:a_hi].numpy(), sc.buf["ts"][b_lo:b_hi].numpy()])
        q.put((rank, sc.src_a, sc.src_b - na_g, a_hi - a_lo, b_hi - b_lo, ts.min() if len(ts) else None,
               ts.max() if len(ts) else None, na_g, sc.n_xchg))
    except Exception as e:
        q.put((rank, repr(e)) + (None,) * 7)
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [3, 8])
def test_exchange_strong_split_slices(world):
    """bench.py --gpus N (strong scaling): each rank generates its own index slice of the
    config's ops (synth.lift_slice_soa); the key-range exchange tiles both branches in
    shard order, moving only the ops at the slice edges."""
    n_total = 20_000 * world
    res = _spawn(_strong_worker, world, (n_total,))
    ea = eb = 0
    for r in range(world):
        _, sa, sb, la, lb, tmin, tmax, na_g, nx = res[r]
        assert (sa, sb) == (ea, eb)
        ea, eb = sa + la, sb + lb
        assert nx < 64                            # ops_per_ms = 7: a few ops per edge move
        if r + 1 < world and res[r + 1][5] is not None:
            assert tmax < res[r + 1][5]
    assert ea == na_g and eb == na_g and na_g == world * (n_total // world // 2)


@pytest.mark.parametrize("seed", range(6))
def test_host_cuts_match_full_searches(seed):
    """ShardedCompose._host_cuts (the one-sync plan) gives the cuts a binary search over
    every whole slice gives, or declines (None) when a splitter falls between a slice's
    head and tail keys; slices of 0..3*RH keys, ties across splitters included."""
    from semantic_merge_amd.shard import RH, ShardedCompose
    rng = np.random.default_rng(seed)
    W = int(rng.integers(2, 6))
    sl = [[np.sort(rng.integers(-50, 50, size=int(rng.integers(0, 3 * RH)))).astype(np.int64)
           for _ in range(2)] for _ in range(W)]
    g = np.zeros((W, 9 + 4 * RH), np.int64)
    for q in range(W):
        for br in range(2):
            k = sl[q][br]
            n, h = len(k), min(RH, len(k))
            g[q, br] = n
            o = 9 + 2 * RH * br
            g[q, o: o + h] = k[:h]
            g[q, o + 2 * RH - h: o + 2 * RH] = k[n - h:]
    declined = 0
    for _ in range(20):
        tau = np.sort(rng.integers(-60, 60, size=W - 1)).astype(np.int64)
        got = ShardedCompose._host_cuts(g, tau)
        want = np.zeros((W, 2, W), np.int64)
        for q in range(W):
            for br in range(2):
                c = np.searchsorted(sl[q][br], tau, side="left")
                want[q, br] = np.diff(np.concatenate([[0], c, [len(sl[q][br])]]))
        if got is None:
            declined += 1
            # a decline only when some splitter really falls strictly inside a middle
            assert any(len(k) > RH and k[RH - 1] < t <= k[len(k) - RH]
                       for q in range(W) for k in sl[q] for t in tau)
        else:
            assert np.array_equal(got, want), (tau, got, want)
    assert declined < 20


def test_tab32_bits_within_library_limit():
    """The 32-bit partial tables are used only for worlds whose rank tag fits the limit
    smx_shard_step accepts (tab32 <= 8 bits); larger worlds keep the 64-bit tables."""
    from semantic_merge_amd.shard import TAB32_MAX_BITS, tab32_bits
    assert TAB32_MAX_BITS == 8
    assert tab32_bits(1) == 1 and tab32_bits(8) == 4 and tab32_bits(255) == 8
    assert tab32_bits(256) == 0 and tab32_bits(1 << 14) == 0


def test_range_info_empty_slice_keys_are_zero():
    """The range info's host path (gloo, CPU tensors) reads key 0 for every entry of an
    empty branch slice, as the device kernel k_range_info writes them (tests/test_gpu_shard.py
    pins the device layout)."""
    import torch.distributed as dist
    from semantic_merge_amd import shard
    from semantic_merge_amd.marshal import SoA
    store = _store_path()
    dist.init_process_group("gloo", store=dist.FileStore(store, 1), rank=0, world_size=1)
    try:
        full = _soa(2_000, 5, 64)
        na = full.n_a
        soa = SoA(na, 0, full.kind[:na], full.ts[:na], full.oid_hi[:na], full.oid_lo[:na], full.sym[:na],
                  full.v0[:na], full.v1[:na], full.n_sym)
        a, b, ga, gb = shard.slices_from_soa(soa, 0, 1, "cpu")
        sc = shard.ShardedCompose(a, b, ga, gb, soa.n_sym, shard.Comm(), "cpu", halo_cap=64, mode="auto")
        info = sc._range_info().numpy()
        RH = shard.RH
        assert info[0] == na and info[1] == 0
        assert info[4] == 0 and info[5] == 0                       # B's first / last key
        assert not info[9 + 2 * RH: 9 + 4 * RH].any()              # B's head and tail keys
        assert info[9: 9 + 2 * RH].all()                           # A's are real keys (never 0 here)
    finally:
        dist.destroy_process_group()
        shutil.rmtree(os.path.dirname(store), ignore_errors=True)
