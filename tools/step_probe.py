#!/usr/bin/env python3
"""tools/step_probe.py -- per-step host time of bench.py's voice loops (diagnostic, GPU box).

Runs the voice workload (NoteOn for all at setup, NoteOff for all mid-run) and the voice_events
workload (5 % note events per block) exactly as bench.py's timed loop calls the library, and
prints per step: the host time of the calls, and the GPU time per step from one event pair.
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
    n, B, W, K = 32768, 256, 5, int(os.environ.get("K", "20"))
    res = {}
    for leg in ("voice", "voice_events"):
        e = ofx.Engine("voice", n)
        e.set_params(0, instance_params("voice", 0, n))
        notes = voice_notes(0, n)
        e.note_events(e.make_events(np.arange(n), 1, notes))
        note_off = e.make_events(np.arange(n), 0, notes)
        gi = np.arange(n)
        evs = [np.concatenate([e.make_events(np.nonzero(gi % 40 == k)[0], 1, notes[gi % 40 == k]),
                               e.make_events(np.nonzero(gi % 40 == (k + 20) % 40)[0], 0, 60)]) for k in range(40)]
        stream = torch.cuda.Stream(dev)
        out = torch.empty((1, B, n), device=dev)
        args = (e.handle, ctypes.c_void_p(0), ctypes.c_void_p(out.data_ptr()), B, _lib.IO_DEVICE,
                ctypes.c_void_p(stream.cuda_stream))
        ev_args = [(e.handle, a.ctypes.data_as(ctypes.POINTER(_lib.Event)), len(a)) for a in evs]
        lib = e.lib
        host = []

        def step(k):
            t0 = time.perf_counter()
            if k == W + K // 2:
                lib.olfx_note_events(e.handle, note_off.ctypes.data_as(ctypes.POINTER(_lib.Event)), len(note_off))
            if leg == "voice_events":
                lib.olfx_note_events(*ev_args[k % 40])
            lib.olfx_process(*args)
            host.append((time.perf_counter() - t0) * 1e6)

        for k in range(W):
            step(k)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        host.clear()
        t0 = time.perf_counter()
        a.record(stream)
        for k in range(K):
            step(W + k)
        b.record(stream)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / K * 1e6
        res[leg] = {"gpu_us_per_step": a.elapsed_time(b) / K * 1e3, "wall_us_per_step": wall,
                    "host_us_per_step_median": float(np.median(host)), "host_us_max": float(np.max(host)),
                    "host_us": [round(h, 1) for h in host]}
        e.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
