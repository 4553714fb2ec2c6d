"""Diagnostic (round 2): per-role busy / waiting cycles of chain_block_v4, from a build with
-DOLFX_CHAIN_STAMP (each wave writes [total cycles, cycles inside wait_for] into its workgroup's
first output slots; the outputs are garbage in that build).  Usage:
  OLFX_LIB=build/ab/stamp.so python tools/chain_stamps.py [instances]"""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
import ol_dsp_amd as ofx

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
e = ofx.Engine("chain", n)
x = (torch.rand((2, 256, n), device="cuda") - 0.5)
for _ in range(4):
    y = e.process(x)
torch.cuda.synchronize()
y = y.cpu().numpy()
wg = np.arange(0, n, 64)
for w, name in enumerate(["C0", "C1", "P", "DT"]):
    tot, wait = y[0, w, wg], y[0, w, wg + 1]
    print(f"{name}: total {tot.mean():.0f} cyc, waiting {wait.mean():.0f} ({100 * wait.mean() / tot.mean():.1f} %)")
