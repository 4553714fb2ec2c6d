"""Diagnostic: does a libolfx kernel launch from a torch process produce output?"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ol_dsp_amd as ofx  # noqa: E402

dev = torch.device("cuda:0")
n = 64
x = np.zeros((2, 256, n), np.float32)
x[:, 0, :] = 1.0
e = ofx.Engine("dattorro", n)
yh = e.process(x)                                   # host path, engine stream
print("host path: nonzero", int(np.count_nonzero(yh)), "sum", float(np.abs(yh).sum()))
e.sync()
e2 = ofx.Engine("dattorro", n)
xd = torch.from_numpy(x).to(dev)
out = torch.full((2, 256, n), 7.0, device=dev)
e2.process(xd, out=out, stream=0)                   # device pointers, engine stream
e2.sync()
print("device path engine stream: nonzero", int((out != 0).sum()), "sevens", int((out == 7).sum()))
e3 = ofx.Engine("dattorro", n)
out3 = torch.full((2, 256, n), 7.0, device=dev)
e3.process(xd, out=out3)                            # torch stream
torch.cuda.synchronize()
e3.sync()
print("device path torch stream: nonzero", int((out3 != 0).sum()), "sevens", int((out3 == 7).sum()))
print("maps:")
for line in open("/proc/self/maps"):
    if "amdhip" in line or "hsa-runtime" in line:
        print("  ", line.split()[-1])
