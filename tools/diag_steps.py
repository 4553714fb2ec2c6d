"""Diagnostic: where does the wall time per bench step go beyond the kernel?  Times 200 chorus
steps (a) as bench.py does (two events per step), (b) without events, (c) the host loop alone
(no GPU wait), and (d) with the launches captured once in a HIP graph and replayed."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ol_dsp_amd as ofx  # noqa: E402
from bench import draw_params  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "chorus"
n = {"chorus": 65536, "dattorro": 65536, "fxrack": 65536, "chain": 16384, "voice": 32768}[wl]
dev = torch.device("cuda:0")
e = ofx.Engine(wl, n, block=256)
e.set_params(0, draw_params(wl, n, 1))
ich = e.info.in_channels
pool = [torch.rand((ich, 256, n), device=dev) - 0.5 for _ in range(8)] if ich else [None]
out = torch.empty((e.info.out_channels, 256, n), device=dev)
s = torch.cuda.Stream(dev)
K = 200


def run(events):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        if events:
            ev[k][0].record(s)
        e.process(pool[k % len(pool)], out=out, n_frames=256, stream=s.cuda_stream)
        if events:
            ev[k][1].record(s)
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    km = sum(a.elapsed_time(b) for a, b in ev) / K if events else float("nan")
    return t / K * 1e3, t_host / K * 1e3, km


for k in range(20):
    e.process(pool[k % len(pool)], out=out, n_frames=256, stream=s.cuda_stream)
for name, evs in (("events", True), ("no events", False), ("events", True), ("no events", False)):
    ms, host_ms, km = run(evs)
    print(f"{wl} {name:10s}: wall {ms:.4f} ms/step, host loop {host_ms:.4f} ms/step, kernel {km:.4f} ms")
