#!/usr/bin/env python3
"""tools/ctl_probe.py -- host-side cost of the control path, per call (diagnostic, GPU box).

Times (perf_counter, no device sync inside the loop) each library call of a control leg: the
parameter / event call and olfx_process, for the voice with 5 % note events per block and the
chain with one scattered parameter on 1 % of the instances per block.  Prints one JSON line.
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
    res = {}
    for kind, n in (("voice", 32768), ("chain", 16384)):
        e = ofx.Engine(kind, n)
        e.set_params(0, instance_params(kind, 0, n))
        lib = e.lib
        stream = torch.cuda.Stream(dev)
        ich = e.info.in_channels
        x = torch.zeros((max(ich, 1), 256, n), device=dev)
        out = torch.empty((e.info.out_channels, 256, n), device=dev)
        args = (e.handle, ctypes.c_void_p(x.data_ptr() if ich else 0), ctypes.c_void_p(out.data_ptr()), 256,
                _lib.IO_DEVICE, ctypes.c_void_p(stream.cuda_stream))
        notes = voice_notes(0, n)
        gi = np.arange(n)
        evs = [np.concatenate([e.make_events(np.nonzero(gi % 40 == k)[0], 1, notes[gi % 40 == k]),
                               e.make_events(np.nonzero(gi % 40 == (k + 20) % 40)[0], 0, 60)]) for k in range(40)]
        sel = [np.ascontiguousarray(np.nonzero(gi % 100 == k)[0].astype(np.uint32)) for k in range(100)]
        vals = [np.full(len(s), 0.3 + 0.001 * k, np.float32) for k, s in enumerate(sel)]
        t_ctl, t_proc, t_plain = [], [], []
        for k in range(60):
            t0 = time.perf_counter()
            if kind == "voice":
                ev = evs[k % 40]
                rc = lib.olfx_note_events(e.handle, ev.ctypes.data_as(ctypes.POINTER(_lib.Event)), len(ev))
            else:
                s_, v_ = sel[k % 100], vals[k % 100]
                rc = lib.olfx_set_param_list(e.handle, 5, s_.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                             v_.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), len(s_))
            t1 = time.perf_counter()
            rc |= lib.olfx_process(*args)
            t2 = time.perf_counter()
            assert rc == 0
            if k >= 10:
                t_ctl.append(t1 - t0)
                t_proc.append(t2 - t1)
        torch.cuda.synchronize()
        for k in range(60):
            t1 = time.perf_counter()
            lib.olfx_process(*args)
            t2 = time.perf_counter()
            if k >= 10:
                t_plain.append(t2 - t1)
        torch.cuda.synchronize()
        res[kind] = {"ctl_call_us": 1e6 * float(np.median(t_ctl)), "process_with_ctl_us": 1e6 * float(np.median(t_proc)),
                     "process_with_ctl_max_us": 1e6 * float(np.max(t_proc)),
                     "process_plain_us": 1e6 * float(np.median(t_plain))}
        e.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
