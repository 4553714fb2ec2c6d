"""Instance sharding across GPUs, the rank launcher and the single end-of-run reduction
(SURVEY.md section 8e).

Every effect instance is an independent recurrence, so the multi-GPU layout is a contiguous
instance range per rank (one process per GPU, one engine per process) with NO collective in the
data path.  The only communication is one all-reduce after the timed region (RCCL over xGMI on
MI355X via the "nccl" backend; gloo in CPU tests): max of the elapsed times, sum of the frames
processed, sum of per-rank output checksums, sum of the ranks that reported.

`launch_ranks` is the torchrun-equivalent used by `bench.py --gpus N` when no launcher set
WORLD_SIZE: it starts N child processes of the same command, one per GPU, BEFORE the parent has
touched the GPU, each with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time
from dataclasses import dataclass
from typing import List, Sequence, Tuple


@dataclass
class RunStats:
    elapsed_s: float     # wall time of the timed region (max over ranks after reduce)
    kernel_ms: float     # mean launch duration of the dominant kernel (max over ranks)
    frames: float        # instance-frames processed (sum over ranks)
    checksum: float      # sum |y| over the last output block (sum over ranks)
    ranks: float = 1.0   # ranks that reported (sum over ranks)


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
    """One all-reduce of the run counters (no-op when torch.distributed is not initialised).  A
    process group of world size 1 (a launcher's single rank) runs the collective too, so the RCCL
    path is exercised on a one-GPU box exactly as at N > 1 (tests/test_gpu_rccl.py)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return stats
    t_max = torch.tensor([stats.elapsed_s, stats.kernel_ms], dtype=torch.float64, device=device)
    t_sum = torch.tensor([stats.frames, stats.checksum, stats.ranks], dtype=torch.float64, device=device)
    dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    dist.all_reduce(t_sum, op=dist.ReduceOp.SUM)
    return RunStats(float(t_max[0]), float(t_max[1]), float(t_sum[0]), float(t_sum[1]), float(t_sum[2]))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(argv: Sequence[str], world: int, poll_s: float = 0.2) -> int:
    """Run `argv` as `world` rank processes (one per GPU) and return the worst exit code.

    The parent never initialises the GPU (it must not: a process that has, may not exec another
    program on the GPU box); each child reads its rank from the environment exactly as under
    `torch.distributed.run`.  If a rank fails, the others are stopped (their own PIDs only) so
    that none waits forever in a collective.  Rank 0 alone prints the result line."""
    port = free_port()
    procs: List[subprocess.Popen] = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world),
                   LOCAL_WORLD_SIZE=str(world), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen(list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0:
                rc = rc or code
                for q in live:          # a failed rank: stop the rest rather than hang in a barrier
                    q.terminate()
        time.sleep(poll_s)
    for p in procs:
        code = p.wait()
        if code != 0 and rc == 0:
            rc = code
    return rc if rc >= 0 else 128 - rc


def self_command() -> List[str]:
    """The command line that started this Python program, for launch_ranks."""
    return [sys.executable, "-u"] + list(sys.argv)
