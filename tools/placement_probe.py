#!/usr/bin/env python3
"""tools/placement_probe.py -- does a workload's kernel time depend on where its memory lands?
Creates <engines> engines of one workload in ONE process (all kept alive, so each gets fresh device
memory), each with its own input pool, and times each over <regions> regions of <steps> steps after
50 warm-up steps (HIP events on the engine's stream).  mode "engines": a new engine and input pool
each time; "pool": one input pool for every engine (a new engine only); "onepool": one engine, a new
input pool each time.  Usage (GPU box):
    python tools/placement_probe.py <workload> <instances> [engines] [mode]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import bench
    import ol_dsp_amd as ofx
    from ol_dsp_amd.workload import instance_params, noise_torch

    name, n = sys.argv[1], int(sys.argv[2])
    engines = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    mode = sys.argv[4] if len(sys.argv) > 4 else "engines"
    steps, regions = 40, 3
    kind = bench.WORKLOADS[name][0]
    dev = torch.device("cuda", 0)
    B = 256
    keep = []
    eng = pool = None
    for k in range(engines):
        if eng is None or mode != "onepool":
            eng = ofx.Engine(kind, n, sample_rate=48000.0, block=B, device=0)
            eng.set_params(0, instance_params(bench.PARAM_SET.get(name, kind), 0, n))
        ich, och = eng.info.in_channels, eng.info.out_channels
        pool_n = max(2, int(1.0e9 // (ich * B * n * 4)))
        if pool is None or mode != "pool":
            pool = noise_torch(0, n, B, ich, dev, blocks=pool_n)
        out = torch.empty((och, B, n), device=dev)
        keep.append((eng, pool, out))
        s = torch.cuda.current_stream()
        for i in range(50):
            eng.process(pool[i % pool_n], out)
        ms = []
        for r in range(regions):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(s)
            for i in range(steps):
                eng.process(pool[(50 + r * steps + i) % pool_n], out)
            e1.record(s)
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1) / steps)
        print(f"{name} n={n} {mode} {k}: ms/step {np.median(ms):.4f}  regions {[round(m, 4) for m in ms]}", flush=True)


if __name__ == "__main__":
    main()
