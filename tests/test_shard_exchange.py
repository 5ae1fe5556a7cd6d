"""Sharded merge, host side on CPU (gloo, 2-3 ranks): the key-range all-to-all puts every
op on the shard owning its timestamp, in place (headroom), with the global source offsets
the kernels need; the originals come back for the next step.  The compute steps need a
GPU (tests/test_gpu_shard.py)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _soa(n, seed, ops_per_ms):
    from semantic_merge_amd import synth
    return synth.lift_soa(synth.lift_logs(synth.LiftSpec(n, 50, seed, ops_per_ms=ops_per_ms)))


def _worker(rank, world, port, args, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from semantic_merge_amd import shard
        n, seed, opm, headroom = args
        soa = _soa(n, seed, opm)
        a, b, na, nb = shard.slices_from_soa(soa, rank, world, "cpu")
        sc = shard.ShardedCompose(a, b, na, nb, soa.n_sym, shard.Comm(), "cpu", halo_cap=64,
                                  headroom=headroom)
        sc.exchange()
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


@pytest.mark.parametrize("world,n,opm,headroom", [(2, 20_000, 64, None), (3, 30_000, 7, None),
                                                  (3, 9_000, 1000, 0)])
def test_exchange_key_ranges(world, n, opm, headroom):
    from semantic_merge_amd import shard
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    args = (n, 3, opm, headroom)
    procs = [ctx.Process(target=_worker, args=(r, world, port, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        item = q.get(timeout=120)
        res[item[0]] = item
    for p in procs:
        p.join(60)
    errs = [res[r][1] for r in range(world) if isinstance(res[r][1], str)]
    assert not errs, errs
    soa = _soa(n, 3, opm)
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
