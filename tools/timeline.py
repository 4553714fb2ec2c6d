#!/usr/bin/env python3
"""tools/timeline.py -- summarise a rocprofv3 --kernel-trace --hip-trace run (diagnostic):
mean host duration per HIP API call, and the gaps between consecutive kernels of one name.
Usage: python tools/timeline.py <rocprof output dir> [kernel substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict

import numpy as np

d = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "voice_block"
api = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)
ker = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
if api:
    acc = defaultdict(list)
    with open(api[0]) as f:
        for r in csv.DictReader(f):
            acc[r["Function"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = sorted(acc.items(), key=lambda kv: -sum(kv[1]))[:15]
    for name, v in rows:
        print(f"api {name:40s} n={len(v):6d} mean={np.mean(v):9.2f} us  p50={np.median(v):8.2f}  total={sum(v)/1e3:8.2f} ms")
if ker:
    ks = []
    with open(ker[0]) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ks.sort()
    sel = [k for k in ks if kname in k[2]]
    dur = [(b - a) / 1e3 for a, b, _ in sel]
    gaps = [(sel[i + 1][0] - sel[i][1]) / 1e3 for i in range(len(sel) - 1)]
    print(f"kernel {kname}: n={len(sel)} mean dur {np.mean(dur):.2f} us; gap to next: mean {np.mean(gaps):.2f} p50 {np.median(gaps):.2f} us")
    print("last 12 (dur, gap):", [(round(a, 1), round(g, 1)) for a, g in zip(dur[-12:], gaps[-12:])])
