#!/usr/bin/env python3
"""Diagnostic (GPU box): where does the fused chain leave the composed oracle on a long run?
Runs the chain, the standalone chorus / pitch-shift / reverb engines and the oracle on the same
inputs under several block schedules and prints the first mismatching (ch, frame, instance)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import torch
import oracle as O
import ol_dsp_amd as ofx
from helpers import chorus_params, dt_params, fast_noise, first_mismatch

cuda = torch.device("cuda:0")


def run(e, x, blocks):
    outs, f0 = [], 0
    for b in blocks:
        xb = torch.from_numpy(np.ascontiguousarray(x[:, f0:f0 + b])).to(cuda)
        outs.append(e.process(xb).cpu().numpy()); f0 += b
    return np.concatenate(outs, 1)


def fm(a, b):
    r = first_mismatch(a, b)
    return "equal" if r is None else f"first mismatch {r[0]} of {r[3]}"


n, frames = 100, int(sys.argv[1]) if len(sys.argv) > 1 else 16384
rng = np.random.default_rng(41)
pc, pp, pd = chorus_params(rng, n), chorus_params(rng, n)[[0, 7]], dt_params(rng, n, 0.0)
pd[0] = rng.uniform(0, 1, n)
x = fast_noise(n, frames, seed=41)
c1, c2, d = O.Chorus(n), O.Chorus(n, mode=1), O.Dattorro(n)
for i in range(n):
    for f in range(8):
        c1.set(i, f, float(pc[f, i]))
    c2.set(i, "pitch", float(pp[0, i])); c2.set(i, "window", float(pp[1, i]))
    for f in range(7):
        d.set(i, f, float(pd[f, i]))
yc = c1.process(x); yp = c2.process(yc); yr = d.process(yp)
for blocks in ([256] * (frames // 256), [4096] * (frames // 4096)):
    tag = f"blocks {blocks[0]}"
    e = ofx.Engine("chorus", n); e.set_params(0, pc); gc = run(e, x, blocks)
    print(tag, "chorus  vs oracle:", fm(gc, yc))
    e = ofx.Engine("pitchshift", n); e.set_params(0, pp); gp = run(e, yc, blocks)
    print(tag, "pitch   vs oracle:", fm(gp, yp))
    e = ofx.Engine("dattorro", n); e.set_params(0, pd); gd = run(e, yp, blocks)
    print(tag, "reverb  vs oracle:", fm(gd, yr))
    e = ofx.Engine("chain", n); e.set_params(0, np.concatenate([pc, pp, pd], 0)); g = run(e, x, blocks)
    print(tag, "chain   vs oracle:", fm(g, yr))
