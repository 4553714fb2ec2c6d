"""Diagnostic: per-phase cycles of chorus_block_v11 from the stamp build (tools/chorus_stamp_build.py).
Usage (GPU box): OLFX_LIB=$PWD/build/ab/chstamp.so python tools/chorus_stamps.py [instances]"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import ol_dsp_amd as ofx  # noqa: E402
from ol_dsp_amd.workload import instance_params  # noqa: E402

PHASES = ["loop", "stageC", "stageAB", "prefetch", "pitch", "psvwin", "st_psv", "chorus", "out", "st_x", "st_plan",
          "st_lines"]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
e = ofx.Engine("chorus", n)
e.set_params(0, instance_params("chorus", 0, n))
x = (torch.rand((2, 256, n), device="cuda") - 0.5)
rows = []
for b in range(6):
    y = e.process(x)
    torch.cuda.synchronize()
    if b >= 2:
        rows.append(y[0, :len(PHASES), 0::32].cpu().numpy().astype(np.float64))
a = np.mean(rows, axis=0)            # [phase][wave]
tot = a.sum(axis=0)
print(f"{n} instances, {a.shape[1]} waves, 16 chunks per wave; cycles per wave per launch (s_memtime units)")
for k, name in enumerate(PHASES):
    print(f"  {name:9s} {a[k].mean():12.0f}  ({100 * a[k].mean() / tot.mean():5.1f} %)  per chunk {a[k].mean() / 16:9.0f}")
print(f"  total     {tot.mean():12.0f}   min {tot.min():.0f} max {tot.max():.0f}")
