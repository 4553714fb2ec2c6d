#!/usr/bin/env python3
"""Summarise tools/pmc_profile.sh output: per-launch counter averages for the dominant kernel,
and the HBM traffic per launch with the gfx950 corrections of MI355X_MICROARCH.md section HBM:
  FETCH_SIZE reads 1/2 of the bytes of a wide coalesced streaming read -> x2 (read side);
  WRITE_SIZE reads exact for 16-B streaming stores.
Both are in KB (rocprofv3 derived counters).  Usage:
  python tools/pmc_traffic.py <workload> <instances> <block> [kernel-substring] [--fetch-scale X] [--out json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, kernel_sub):
    """{kernel: {counter: [per-dispatch values]}} for kernels whose name contains kernel_sub
    (or one of its "|"-separated alternatives)."""
    subs = kernel_sub.split("|")
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", "")
                if not any(x in k for x in subs):
                    continue
                vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return vals


def main():
    wl, n, block = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    ksub = sys.argv[4] if len(sys.argv) > 4 and not sys.argv[4].startswith("--") else "_block_"
    out = None
    if "--out" in sys.argv:
        out = sys.argv[sys.argv.index("--out") + 1]
    # FETCH_SIZE correction: x2 for wide coalesced streaming reads (MI355X_MICROARCH.md), x1 for
    # the chorus' 96-B segment reads -- calibrated per kernel against its known staged bytes
    # 
    fscale = float(sys.argv[sys.argv.index("--fetch-scale") + 1]) if "--fetch-scale" in sys.argv else 2.0
    base = os.path.join("gpurun_out", f"pmc_{wl}")
    agg, res_k = {}, {}
    for p in sorted(glob.glob(os.path.join(base, "p*"))):
        if not os.path.isdir(p):
            continue
        # counter rows are per dispatch (already summed over XCDs by rocprofv3); one engine call
        # launches each matching kernel once (the chain launches three), so per launch =
        # the sum over kernels of each kernel's per-dispatch mean
        for kern, cnt in load(p, ksub).items():
            for k, v in cnt.items():
                agg[k] = agg.get(k, 0.0) + sum(v) / len(v)
                res_k.setdefault(kern.split("(")[0], {})[k] = sum(v) / len(v)
    for k in sorted(agg):
        print(f"{k:28s} {agg[k]:.6g}")
    res = {"workload": wl, "instances": n, "block": block, "counters_per_launch": agg,
           "counters_per_kernel": res_k}
    # the build the counters were taken with (tools/pmc_profile.sh): bench.py refuses a traffic file
    # whose libolfx.so hash differs from the library it runs
    stamp = os.path.join(base, "libolfx.sha256")
    if not os.path.exists(stamp):
        sys.exit(f"{stamp} missing: re-run tools/pmc_profile.sh (it records the library's hash)")
    with open(stamp) as f:
        res["libolfx_sha256"] = f.read().split()[0]
    if "FETCH_SIZE" in agg and "WRITE_SIZE" in agg:
        fetch = agg["FETCH_SIZE"] * 1024 * fscale
        write = agg["WRITE_SIZE"] * 1024
        res.update({"fetch_bytes_corrected": fetch, "write_bytes": write,
                    "hbm_bytes_per_launch": fetch + write,
                    "hbm_bytes_per_frame": (fetch + write) / (n * block),
                    "fetch_scale": fscale,
                    "note": f"FETCH_SIZE x{fscale:g} (per-kernel calibration, DESIGN.md section 5) + WRITE_SIZE"})
        print(f"HBM bytes/launch {fetch + write:.4g}  per frame {(fetch + write) / (n * block):.2f}")
    # request-size accounting: the L2's memory-side read/write requests by size (gfx950 has 32-,
    # 64- and 128-B read requests; RDREQ counts requests of every size)
    if all(k in agg for k in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum",
                              "TCC_EA0_RDREQ_128B_sum")):
        r32, r64, r128 = agg["TCC_EA0_RDREQ_32B_sum"], agg["TCC_EA0_RDREQ_64B_sum"], agg["TCC_EA0_RDREQ_128B_sum"]
        rd = 32 * r32 + 64 * r64 + 128 * r128
        res["read_bytes_by_request_size"] = rd
        res["read_requests_other"] = agg["TCC_EA0_RDREQ_sum"] - r32 - r64 - r128
        print(f"read bytes by request size {rd:.4g} (per frame {rd / (n * block):.2f}); "
              f"unsized requests {res['read_requests_other']:.4g}")
    if "TCC_EA0_WRREQ_sum" in agg and "TCC_EA0_WRREQ_64B_sum" in agg:
        w64 = agg["TCC_EA0_WRREQ_64B_sum"]
        wr = 64 * w64 + 32 * (agg["TCC_EA0_WRREQ_sum"] - w64)
        res["write_bytes_by_request_size"] = wr
        print(f"write bytes by request size {wr:.4g} (per frame {wr / (n * block):.2f})")
        if "read_bytes_by_request_size" in res:    # preferred: no width calibration needed
            tot = res["read_bytes_by_request_size"] + wr
            res.update({"hbm_bytes_per_launch": tot, "hbm_bytes_per_frame": tot / (n * block),
                        "method": "TCC_EA0_RDREQ_{32B,64B,128B} x size + TCC_EA0_WRREQ(_64B) x size; "
                                  "FETCH_SIZE x fetch_scale + WRITE_SIZE kept as the cross-check"})
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
