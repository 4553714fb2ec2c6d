#!/usr/bin/env python3
"""Per-launch averages of tools/pmc_util.sh counters for the dominant kernel of each workload.
Usage: python tools/pmc_util_summary.py <workload> [kernel-substring]"""
import csv, glob, os, sys
from collections import defaultdict

wl = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "_block"
vals = defaultdict(list)
for f in glob.glob(f"gpurun_out/util_{wl}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
# rows are per dispatch (values already summed over dimensions by rocprofv3) -- average them
avg = {k: sum(v) / len(v) for k, v in vals.items()}
for k in sorted(avg):
    print(f"{k:36s} {avg[k]:16.1f}")
g = avg.get("GRBM_GUI_ACTIVE")
if g:
    # GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles (≈ 8 x the kernel's cycles); the _sum counters sum
    # 256 per-CU units: the average unit's busy fraction is (sum / 256) / (GRBM / 8)
    for k in ("TA_TA_BUSY_sum", "TD_TD_BUSY_sum", "TCP_PENDING_STALL_CYCLES_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum"):
        if k in avg:
            print(f"{k} / GRBM_GUI_ACTIVE = {avg[k] / g:.1f}  -> per-CU unit busy fraction {avg[k] / g * 8 / 256:.2f}")
if "SQ_WAVE_CYCLES" in avg:
    wc = avg["SQ_WAVE_CYCLES"]
    for k in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
        if k in avg:
            print(f"{k} / SQ_WAVE_CYCLES = {avg[k] / wc:.3f}")
if "TCC_HIT_sum" in avg:
    print(f"L2 hit rate = {avg['TCC_HIT_sum'] / (avg['TCC_HIT_sum'] + avg['TCC_MISS_sum']):.3f}")
if "TCP_TCC_READ_REQ_sum" in avg:
    print(f"mean L2 read latency (cycles) = {avg['TCP_TCC_READ_REQ_LATENCY_sum'] / avg['TCP_TCC_READ_REQ_sum']:.0f}")
