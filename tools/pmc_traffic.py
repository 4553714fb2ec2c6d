#!/usr/bin/env python3
"""Summarise tools/pmc_profile.sh output: per-launch counter averages for the dominant kernel,
and the HBM traffic per launch with the gfx950 corrections of MI355X_MICROARCH.md section HBM:
  FETCH_SIZE reads 1/2 of the bytes of a wide coalesced streaming read -> x2 (read side);
  WRITE_SIZE reads exact for 16-B streaming stores.
Both are in KB (rocprofv3 derived counters).  Usage:
  python tools/pmc_traffic.py <workload> <instances> <block> [kernel-substring] [--out json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, kernel_sub):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel_sub not in row.get("Kernel_Name", ""):
                    continue
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    return vals


def main():
    wl, n, block = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    ksub = sys.argv[4] if len(sys.argv) > 4 and not sys.argv[4].startswith("--") else "_block_"
    out = None
    if "--out" in sys.argv:
        out = sys.argv[sys.argv.index("--out") + 1]
    base = os.path.join("gpurun_out", f"pmc_{wl}")
    agg = {}
    for p in sorted(glob.glob(os.path.join(base, "p*"))):
        if not os.path.isdir(p):
            continue
        for k, v in load(p, ksub).items():
            # counter rows are per dispatch (already summed over XCDs/instances by rocprofv3)
            agg[k] = sum(v) / len(v)
    for k in sorted(agg):
        print(f"{k:28s} {agg[k]:.6g}")
    res = {"workload": wl, "instances": n, "block": block, "counters_per_launch": agg}
    if "FETCH_SIZE" in agg and "WRITE_SIZE" in agg:
        fetch = agg["FETCH_SIZE"] * 1024 * 2.0      # gfx950: FETCH_SIZE = 1/2 of streamed bytes
        write = agg["WRITE_SIZE"] * 1024
        res.update({"fetch_bytes_corrected": fetch, "write_bytes": write,
                    "hbm_bytes_per_launch": fetch + write,
                    "hbm_bytes_per_frame": (fetch + write) / (n * block),
                    "note": "FETCH_SIZE x2 per MI355X_MICROARCH.md (wide streaming reads); "
                            "uncalibrated for 4-B scattered accesses"})
        print(f"HBM bytes/launch {fetch + write:.4g}  per frame {(fetch + write) / (n * block):.2f}")
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
