"""Phase timing of chorus_block_v13 from a -DOLFX_CB_STAMP=1 build (tools/build_variant.sh):
workgroup 0's s_memtime at each phase boundary of each round, for the last of a few blocks.
Usage (GPU box): OLFX_LIB=build/ab/stamp.so python tools/cb_stamps.py [kind] [n]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ol_dsp_amd as ofx  # noqa: E402
from ol_dsp_amd.workload import instance_params, noise_torch  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "chorus"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
e = ofx.Engine(kind, n)
e.set_params(0, instance_params(kind, 0, n))
xs = noise_torch(0, n, 256, 2, torch.device("cuda"), blocks=4)
for x in xs:
    y = e.process(x)
torch.cuda.synchronize()
buf = (ctypes.c_uint64 * 512)()
assert e.lib.olfx_debug_stamps(buf, 512) == 0
st = np.array(buf[:], np.int64)
# layout: 0 start; per round: 1 round start, 2 after p1 + barrier, 3 after issue, [4 after p2], 5 after
# p3 + barrier, [6 after out, 7 after fill] (the last round stops after out)
labels = ["p1+scal", "issue", "p2", "p3+phasors", "out", "fill"] if kind == "chorus" else \
         ["p1+scal", "issue", "p3+phasors", "out", "fill"]
per = len(labels) + 1
t0 = st[0]
rounds = []
k = 1
while k + per <= 500 and st[k + per - 1] > 0:
    rounds.append(np.diff(st[k:k + per]))
    k += per
r = np.array(rounds)
print(f"{kind} n={n}: prologue {st[1] - t0} cycles; {len(r)} full rounds")
print("phase      " + " ".join(f"{l:>11s}" for l in labels))
print("mean cyc   " + " ".join(f"{v:11.0f}" for v in r.mean(0)))
print("round mean", r.sum(1).mean(), "cycles")
