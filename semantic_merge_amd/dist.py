"""Multi-GPU plumbing shared by bench.py and the tests (one process per GPU):
rank info from the torchrun environment, the MAX all-reduce of the elapsed time and the
whole-job throughput.  The sharded merge itself lives in shard.py.  The backend is RCCL
("nccl") on GPUs; the same helpers run on "gloo" in the CPU tests.
"""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass
class RankInfo:
    world: int
    rank: int
    local: int


def rank_info() -> RankInfo:
    return RankInfo(int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
                    int(os.environ.get("LOCAL_RANK", "0")))


def rank_seed(base_seed: int, rank: int) -> int:
    """Each rank's merge uses its own seed: independent logs, same distribution."""
    return base_seed + rank


def max_over_ranks(value: float, device=None) -> float:
    """MAX all-reduce of one float (the job time is the slowest rank's)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    if dist.get_backend() != "nccl":
        device = None  # gloo: host tensor
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def job_throughput(units_per_rank: int, world: int, steps: int, elapsed_max: float) -> float:
    """Whole-job units per second: every rank's units over the slowest rank's time."""
    return world * units_per_rank * steps / elapsed_max
