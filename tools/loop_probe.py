#!/usr/bin/env python3
"""tools/loop_probe.py -- is a short-kernel bench loop host-bound?  (diagnostic, GPU box)

For the voice engine (a ~35 us kernel), times K steps of olfx_process three ways: bare calls,
calls bracketed by two torch timing events (bench.py's loop), and the same after a GPU sleep that
lets the host enqueue every step before the GPU reaches them (the events then see GPU time only).
Prints one JSON line: wall us/step and mean event us/step of each, host us per event record.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import ol_dsp_amd as ofx
    from ol_dsp_amd import _lib
    from ol_dsp_amd.workload import instance_params, voice_notes
    dev = torch.device("cuda:0")
    K = 200
    res = {}
    for kind, n in (("voice", 32768), ("chorus", 65536)):
        e = ofx.Engine(kind, n)
        e.set_params(0, instance_params(kind, 0, n))
        if kind == "voice":
            e.note_events(e.make_events(np.arange(n), 1, voice_notes(0, n)))
        s = torch.cuda.Stream(dev)
        ich = e.info.in_channels
        x = torch.zeros((max(ich, 1), 256, n), device=dev)
        out = torch.empty((e.info.out_channels, 256, n), device=dev)
        args = (e.handle, ctypes.c_void_p(x.data_ptr() if ich else 0), ctypes.c_void_p(out.data_ptr()), 256,
                _lib.IO_DEVICE, ctypes.c_void_p(s.cuda_stream))
        lib = e.lib
        for _ in range(20):
            lib.olfx_process(*args)
        torch.cuda.synchronize()
        r = {}
        # bare
        t0 = time.perf_counter()
        for _ in range(K):
            lib.olfx_process(*args)
        torch.cuda.synchronize()
        r["bare_wall_us"] = (time.perf_counter() - t0) / K * 1e6
        # events, as bench.py
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
        t0 = time.perf_counter()
        th = 0.0
        for a, b in evs:
            t1 = time.perf_counter()
            a.record(s)
            th += time.perf_counter() - t1
            lib.olfx_process(*args)
            b.record(s)
        torch.cuda.synchronize()
        r["events_wall_us"] = (time.perf_counter() - t0) / K * 1e6
        r["events_kernel_us"] = float(np.mean([a.elapsed_time(b) for a, b in evs])) * 1e3
        r["host_us_per_record"] = th / K * 1e6
        # events after a GPU sleep: the host is ahead for every step
        with torch.cuda.stream(s):
            torch.cuda._sleep(int(2e8))
        for a, b in evs:
            a.record(s)
            lib.olfx_process(*args)
            b.record(s)
        torch.cuda.synchronize()
        r["ahead_kernel_us"] = float(np.mean([a.elapsed_time(b) for a, b in evs])) * 1e3
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s):
            torch.cuda._sleep(int(2e8))
        ev0.record(s)
        for _ in range(K):
            lib.olfx_process(*args)
        ev1.record(s)
        torch.cuda.synchronize()
        r["ahead_bare_gpu_us_per_step"] = ev0.elapsed_time(ev1) / K * 1e3
        res[kind] = r
        e.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
