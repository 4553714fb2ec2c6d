"""RCCL on the hardware we have: the multi-GPU bench's only collective -- the
end-of-run reduction of dist.reduce_stats over RCCL/xGMI ("nccl" backend) -- executed on the GPU box
at world size 1, so that the first 8-GPU driver run is not the first RCCL call.

Each case runs in a child process (its own process group; pytest's process keeps no RCCL state),
started as a child, never exec'd, with MASTER_ADDR 127.0.0.1.
"""
import json
import os
import subprocess
import sys

import pytest

from ol_dsp_amd.dist import free_port

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_REDUCE = r"""
import torch, torch.distributed as dist
from ol_dsp_amd.dist import RunStats, reduce_stats
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
s = reduce_stats(RunStats(0.25, 0.125, 3.0e9, 1234.5, 1.0), device=dev)
assert (s.elapsed_s, s.kernel_ms, s.frames, s.checksum, s.ranks) == (0.25, 0.125, 3.0e9, 1234.5, 1.0), s
# a bucket-sized device all-reduce and a max-reduce through the same communicator
x = torch.arange(1 << 20, device=dev, dtype=torch.float32)
dist.all_reduce(x)
m = torch.tensor([7.0, -1.0], device=dev, dtype=torch.float64)
dist.all_reduce(m, op=dist.ReduceOp.MAX)
torch.cuda.synchronize()
assert torch.equal(x, torch.arange(1 << 20, device=dev, dtype=torch.float32)) and m.tolist() == [7.0, -1.0]
dist.barrier()
dist.destroy_process_group()
print("RCCL_OK")
"""


def _env():
    return dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", LOCAL_WORLD_SIZE="1",
                MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), HSA_ENABLE_IPC_MODE_LEGACY="0",
                PYTHONPATH=ROOT)


def test_reduce_stats_over_rccl_world_1():
    """dist.reduce_stats's two all-reduces (MAX, SUM) on device tensors through an initialised
    nccl (RCCL) process group of one rank, plus a 4 MiB all-reduce and a barrier."""
    r = subprocess.run([sys.executable, "-c", _REDUCE], env=_env(), cwd=ROOT, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0 and "RCCL_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])


def test_bench_under_a_launcher_world_1():
    """bench.py as one launcher rank (WORLD_SIZE=1 set): the nccl process group of bench.py:main, the
    barriers around the timed region and reduce_stats over RCCL, then the result line."""
    cmd = [sys.executable, "bench.py", "--gpus", "1", "--workload", "chorus", "--instances", "4096",
           "--steps", "3", "--warmup", "1", "--cpu-seconds", "0", "--also", "", "--full-json", ""]
    r = subprocess.run(cmd, env=_env(), cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-4000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 1 and res["ranks_reporting"] == 1 and res["value"] > 0
    assert res["parity"]["ok"] is True
