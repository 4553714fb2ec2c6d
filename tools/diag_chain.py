"""Diagnose the fused chain against the three standalone GPU engines (known-good) on one input."""
import sys
import numpy as np
import torch
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import ol_dsp_amd as ofx
from helpers import chorus_params, dt_params, fast_noise

n, F = 64, 1024
rng = np.random.default_rng(31)
pc = chorus_params(rng, n); pp = chorus_params(rng, n)[[0, 7]]; pd = dt_params(rng, n, 0.1)
x = torch.from_numpy(fast_noise(n, F, seed=31)).cuda()
e = ofx.Engine("chain", n); e.set_params(0, np.concatenate([pc, pp, pd], 0))
y = torch.cat([e.process(x[:, f:f + 256].contiguous()) for f in range(0, F, 256)], 1)
c1 = ofx.Engine("chorus", n); c1.set_params(0, pc)
c2 = ofx.Engine("pitchshift", n); c2.set_params(0, pp)
d = ofx.Engine("dattorro", n); d.set_params(0, pd)
outs = []
for f in range(0, F, 256):
    a = c1.process(x[:, f:f + 256].contiguous()); b = c2.process(a); outs.append(d.process(b))
yr = torch.cat(outs, 1)
torch.cuda.synchronize()
print("max|y|", y.abs().max().item(), "max|yr|", yr.abs().max().item())
diff = (y != yr)
print("mismatches", int(diff.sum()), "of", diff.numel())
if diff.any():
    idx = torch.nonzero(diff)[0].tolist(); print("first", idx, y[tuple(idx)].item(), yr[tuple(idx)].item())
    per_inst = diff.any(dim=1).any(dim=0)
    print("instances with mismatches", int(per_inst.sum()))
