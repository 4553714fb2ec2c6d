"""Diagnostic (round 4): per-role total and barrier-wait cycles of voice_block_v5, from a build with
-DOLFX_VC_STAMP (each role wave writes [total cycles, cycles at the step barriers] into output
rows 2 role, 2 role + 1; the outputs are garbage in that build).  The stamp code left the kernel in
round 5: build it from the round-4 source, `bash tools/build_variant.sh vcstamp 5fe6fd8 -DOLFX_VC_STAMP=1`.
Usage (GPU box):
  OLFX_LIB=build/ab/vcstamp.so python tools/voice_stamps.py [voices]"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import ol_dsp_amd as ofx  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
e = ofx.Engine("voice", n)
e.note_events([(i, 1, 36 + i % 60) for i in range(n)])
out = torch.empty((1, 256, n), device="cuda")
for _ in range(6):
    e.process(None, out=out)
torch.cuda.synchronize()
y = out.cpu().numpy()[0]
for r, name in enumerate(["ENV", "OSC", "FREQ", "FILT"]):
    tot, wait = y[2 * r], y[2 * r + 1]
    print(f"{name:5s} total {tot.mean():8.0f} cyc  at barriers {wait.mean():8.0f} ({100 * wait.mean() / tot.mean():5.1f} %)  "
          f"busy {tot.mean() - wait.mean():8.0f}")
