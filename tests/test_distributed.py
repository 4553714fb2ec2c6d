"""Multi-process host logic of the multi-GPU path, on CPU with gloo (world_size 2 and 4).

The data path has no collective (instances shard trivially); what is tested
here is the sharding and the single end-of-run reduction bench.py performs over RCCL on GPUs.
"""
import os
import socket

import pytest
import torch.multiprocessing as mp

from ol_dsp_amd.dist import RunStats, reduce_stats, shard


def test_shard_covers_exactly():
    for n in (0, 1, 7, 64, 65536, 262144, 131073):
        for world in (1, 2, 3, 4, 8):
            ranges = [shard(n, world, r) for r in range(world)]
            assert sum(c for _, c in ranges) == n
            pos = 0
            for first, count in ranges:
                assert first == pos and count >= 0
                pos += count
            counts = [c for _, c in ranges]
            assert max(counts) - min(counts) <= 1
    assert shard(262144, 8, 3) == (98304, 32768)     # BASELINE config 4: 32,768 voices / GPU
    assert shard(131072, 8, 7) == (114688, 16384)    # BASELINE config 5: 16,384 chains / GPU
    with pytest.raises(ValueError):
        shard(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, count = shard(65536 * world, world, rank)
    st = RunStats(elapsed_s=1.0 + rank, kernel_ms=0.5 * (rank + 1), frames=float(count * 256),
                  checksum=float(first))
    out = reduce_stats(st)
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def _shard_checksum(first, count):
    """The chorus job's per-shard checksum: the oracle run on this shard's global instances (params
    and inputs from the global index), summed as exact float64 over the output bit patterns."""
    import numpy as np

    import oracle as O
    from ol_dsp_amd.workload import instance_params, noise_np
    p = instance_params("chorus", first, count)
    c = O.Chorus(count)
    for i in range(count):
        for f in range(8):
            c.set(i, f, float(p[f, i]))
    y = c.process(noise_np(first, count, 256, 2))
    return float(y.view(np.uint32).astype(np.float64).sum())


def _worker_job(rank, world, port, n_total, q):
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, count = shard(n_total, world, rank)
    st = RunStats(elapsed_s=1.0, kernel_ms=1.0, frames=float(count * 256), checksum=_shard_checksum(first, count))
    q.put((rank, reduce_stats(st)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_job_checksum_equals_single_rank(world):
    """bench.py's multi-rank layout on CPU: each rank runs the oracle over its shard of a 96-instance
    chorus job, the single all-reduce sums the shard checksums, and the sum equals the one-rank
    job's checksum exactly."""
    n_total = 96
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_job, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    whole = _shard_checksum(0, n_total)
    for _, st in res:
        assert st.checksum == whole
        assert st.frames == n_total * 256


@pytest.mark.parametrize("world", [2, 4])
def test_reduce_stats_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    firsts = sum(shard(65536 * world, world, r)[0] for r in range(world))
    for _, st in res:
        assert st.elapsed_s == 1.0 + (world - 1)              # max over ranks
        assert st.kernel_ms == 0.5 * world
        assert st.frames == 65536 * world * 256                # sum over ranks: whole-job frames
        assert st.checksum == float(firsts)


def test_reduce_stats_single_process_is_identity():
    st = RunStats(2.0, 1.0, 3.0, 4.0)
    assert reduce_stats(st) == st
