#!/usr/bin/env bash
# tools/ab_traffic.sh -- A/B of experimental libolfx.so builds: bench time and L2/EA traffic per
# launch (read requests by size, write requests, L2 hit/miss), one --pmc pass per counter group.
# Usage: bash tools/ab_traffic.sh <workload> <lib> [<lib>...]   ("main" = ol_dsp_amd/libolfx.so)
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
wl=$1; shift
bash tools/ab.sh "$wl" "$@" || exit $?
for lib in "$@"; do
  [ "$lib" = main ] && lib=ol_dsp_amd/libolfx.so
  tag=$(basename "$lib" .so)
  k=0
  for p in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "TCC_HIT_sum TCC_MISS_sum"; do
    k=$((k+1))
    OLFX_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $p -d "gpurun_out/abt_${wl}_$tag/p$k" -o run \
        --output-format csv -- python3 bench.py --workload "$wl" --steps 10 --warmup 2 --cpu-seconds 0 \
        > "gpurun_out/abt_${wl}_${tag}_p$k.log" 2>&1 || { tail -5 "gpurun_out/abt_${wl}_${tag}_p$k.log"; exit 1; }
  done
  python3 - "$wl" "$tag" <<'PY'
import csv, glob, sys
from collections import defaultdict
wl, tag = sys.argv[1], sys.argv[2]
v = defaultdict(list)
for f in glob.glob(f"gpurun_out/abt_{wl}_{tag}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "_block" in r["Kernel_Name"]:
            v[r["Counter_Name"]].append(float(r["Counter_Value"]))
a = {k: sum(x) / len(x) for k, x in v.items()}
frames = {"chorus": 65536, "dattorro": 65536, "fxrack": 65536, "pitchshift": 65536, "chain": 16384}.get(wl, 65536) * 256
rd = a.get("TCC_EA0_RDREQ_128B_sum", 0) * 128 + (a.get("TCC_EA0_RDREQ_sum", 0) - a.get("TCC_EA0_RDREQ_128B_sum", 0)) * 64
wr = a.get("TCC_EA0_WRREQ_64B_sum", 0) * 64 + (a.get("TCC_EA0_WRREQ_sum", 0) - a.get("TCC_EA0_WRREQ_64B_sum", 0)) * 32
hit = a.get("TCC_HIT_sum", 0) / max(1, a.get("TCC_HIT_sum", 0) + a.get("TCC_MISS_sum", 0))
print(f"{wl:10s} {tag:24s} read {rd / frames:6.1f} B/frame  write {wr / frames:6.1f} B/frame  L2 hit {hit:.3f}")
PY
done
