"""Multi-process path of bench.py on CPU: world_size 2 over gloo (127.0.0.1)."""
import os
import shutil
import tempfile

import pytest
import torch.multiprocessing as mp

from semantic_merge_amd import dist as smx_dist


def _worker(rank, world, store_path, q):
    import torch.distributed as dist
    os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank))
    # FileStore rendezvous: no bound-then-freed port for the children to race for
    dist.init_process_group("gloo", store=dist.FileStore(store_path, world), rank=rank, world_size=world)
    info = smx_dist.rank_info()
    dist.barrier()
    elapsed = smx_dist.max_over_ranks(1.0 + rank)  # rank 1 is the slowest
    from semantic_merge_amd import synth
    spec = synth.LiftSpec(2000, 20, smx_dist.rank_seed(11, info.rank))
    soa = synth.lift_soa(synth.lift_logs(spec))
    q.put((info.rank, info.world, elapsed, int(soa.oid_hi[0])))
    dist.destroy_process_group()


def test_two_rank_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    tmp = tempfile.mkdtemp(prefix="smx_store_")
    procs = [ctx.Process(target=_worker, args=(r, 2, os.path.join(tmp, "store"), q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    shutil.rmtree(tmp, ignore_errors=True)
    res = sorted(q.get(timeout=5) for _ in range(2))
    assert [r[0] for r in res] == [0, 1] and all(r[1] == 2 for r in res)
    assert all(r[2] == 2.0 for r in res)            # MAX over ranks seen by every rank
    assert res[0][3] != res[1][3]                   # independent merges per rank
    assert smx_dist.job_throughput(100, 2, 10, 2.0) == pytest.approx(1000.0)
