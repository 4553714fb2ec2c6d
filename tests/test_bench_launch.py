"""bench.py's own rank launcher (`--gpus N` without torchrun), on CPU.

The driver may run `python bench.py --gpus 8` without a launcher; bench.py must then start the
eight rank processes itself (ol_dsp_amd.dist.launch_ranks) before anything touches the GPU.  The
`--stub` leg stands in for the GPU work (gloo, no engine) and goes through the same sharding, the
same single all-reduce and the same rank-0 JSON line as a real leg.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(*args, timeout=180):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout          # exactly one line: rank 0's
    return json.loads(lines[0])


@pytest.mark.parametrize("world", [2, 3])
def test_gpus_n_launches_n_ranks(world):
    n, steps = 1000, 5
    res = _run_bench("--stub", "--gpus", str(world), "--steps", str(steps), "--warmup", "0",
                     "--instances", str(n), "--full-json", "")
    assert res["n_gpus"] == world
    assert res["ranks_reporting"] == world                    # every rank ran and reported
    assert res["frames"] == world * n * 256 * steps           # the shards' sum: the whole job
    assert res["config"]["instances_total"] == world * n
    # the checksum leg sums each rank's shard start: proves the ranks took distinct shards
    from ol_dsp_amd.dist import shard
    assert res["output_checksum"] == sum(shard(world * n, world, r)[0] for r in range(world))
    assert res["scaling"] == "weak"


def test_gpus_1_runs_in_process():
    res = _run_bench("--stub", "--steps", "3", "--warmup", "0", "--instances", "64", "--full-json", "")
    assert res["n_gpus"] == 1 and res["ranks_reporting"] == 1
    assert res["frames"] == 64 * 256 * 3


def test_gpus_4_end_to_end_with_legs():
    """`bench.py --gpus 4` under gloo through the whole flow a GPU run takes: four
    rank processes, two legs kept alive and interleaved over the repetitions (rotated order), one
    all-reduce per region, rank 0's final line.  The line's value is the job's frames summed over
    the four ranks divided by the median region's time (max over ranks)."""
    n, steps, reps = 4096, 4, 3
    res = _run_bench("--stub", "--gpus", "4", "--steps", str(steps), "--warmup", "0", "--leg-warmup", "0",
                     "--reps", str(reps), "--instances", str(n), "--also", "chain", "--full-json", "", timeout=240)
    assert res["n_gpus"] == 4
    assert res["ranks_reporting"] == 4
    assert res["config"]["instances_per_gpu"] == n
    assert res["config"]["instances_total"] == 4 * n
    assert res["frames"] == 4 * n * 256 * steps                 # one region of every rank's shard
    elapsed = res["ms_per_step"] * steps / 1e3                   # the median region (max over ranks)
    assert abs(res["value"] - res["frames"] / elapsed) <= 1e-6 * res["value"]
    assert res["reps"]["n"] == reps and len(res["reps"]["kernel_ms"]) == reps
    leg = res["also"]["chain_16384"]
    assert leg["ranks"] == 4 and leg["n"] == 16384
    from ol_dsp_amd.dist import shard
    assert res["output_checksum"] == sum(shard(4 * n, 4, r)[0] for r in range(4))
