"""Instance sharding across GPUs and the single end-of-run reduction.

Every effect instance is an independent recurrence, so the multi-GPU layout is a contiguous
instance range per rank (one process per GPU, one engine per process) with NO collective in the
data path.  The only communication is one all-reduce after the timed region (RCCL over xGMI on
MI355X via the "nccl" backend; gloo in CPU tests): max of the elapsed times, sum of the frames
processed, sum of per-rank output checksums.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Tuple


@dataclass
class RunStats:
    elapsed_s: float     # wall time of the timed region (max over ranks after reduce)
    kernel_ms: float     # mean launch duration of the dominant kernel (max over ranks)
    frames: float        # instance-frames processed (sum over ranks)
    checksum: float      # sum |y| over the last output block (sum over ranks)


def env_ranks() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment (defaults: single process)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous instance range [first, first+count) of `rank`: GPU g gets [g N/G, (g+1) N/G)."""
    if world <= 0 or not 0 <= rank < world or n_total < 0:
        raise ValueError("bad shard arguments")
    first = (n_total * rank) // world
    last = (n_total * (rank + 1)) // world
    return first, last - first


def reduce_stats(stats: RunStats, device=None) -> RunStats:
    """One all-reduce of the run counters (no-op when torch.distributed is not initialised)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return stats
    t_max = torch.tensor([stats.elapsed_s, stats.kernel_ms], dtype=torch.float64, device=device)
    t_sum = torch.tensor([stats.frames, stats.checksum], dtype=torch.float64, device=device)
    dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    dist.all_reduce(t_sum, op=dist.ReduceOp.SUM)
    return RunStats(float(t_max[0]), float(t_max[1]), float(t_sum[0]), float(t_sum[1]))
