#!/usr/bin/env python3
"""tools/cpu_calibration.py -- BASELINE.md section 3's calibration, run in the build container only:
the real reference reverb (libs/dattorro-verb/verb.cpp compiled here into oracle/_ref) timed next
to the restatement (oracle/dattorro_ref.c) on the same cores, through bench.py's own CPU-baseline
harness (same instances, parameters, xorshift inputs, 256-frame blocks, OpenMP schedule(static)
over instances).  They must agree within +-10 % in speed and be bit-identical in output.

Test infrastructure: it loads oracle/ only (never the product).  Usage:
  python tools/cpu_calibration.py [--threads 8] [--seconds 6] [--out profiles/r3/cpu_calibration.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import oracle as O
    import bench
    from ol_dsp_amd.workload import noise_np
    if not O.ref_available():
        raise SystemExit("oracle/_ref not built (make -C oracle; needs /root/reference)")
    n, block = 8192, 256
    x = noise_np(0, n, block, 2)
    # bit identity over several blocks (state carried), same parameters as the bench
    ref_step, ref_keep = bench._cpu_bank("dattorro", n, 48000.0, False, True)
    port_step, port_keep = bench._cpu_bank("dattorro", n, 48000.0, False, False)
    same = True
    for _ in range(4):
        a, b = ref_step(x, args.threads), port_step(x, args.threads)
        same = same and np.array_equal(np.asarray(a).view(np.uint32), np.asarray(b).view(np.uint32))

    def rate(step):
        step(x, args.threads)
        t0 = time.perf_counter()
        blocks = 0
        while time.perf_counter() - t0 < args.seconds:
            step(x, args.threads)
            blocks += 1
        return blocks * block * n / (time.perf_counter() - t0)

    rr, rp = [], []
    for _ in range(args.rounds):              # interleaved, so drift in the host's load hits both
        rr.append(rate(ref_step))
        rp.append(rate(port_step))
    ref_v, port_v = float(np.median(rr)), float(np.median(rp))
    res = {"what": "dattorro reverb, CPU: reference verb.cpp (oracle/_ref) vs restatement (oracle/dattorro_ref.c)",
           "instances": n, "block": block, "threads": args.threads, "seconds_per_run": args.seconds,
           "reference_samples_per_s": ref_v, "restatement_samples_per_s": port_v,
           "restatement_over_reference": port_v / ref_v, "within_10pct": abs(port_v / ref_v - 1.0) <= 0.10,
           "bit_identical_4_blocks": bool(same), "runs_reference": rr, "runs_restatement": rp,
           "flags": "-O2 -ffp-contract=off (both)"}
    res.update(bench.host_facts())
    print(json.dumps(res, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
