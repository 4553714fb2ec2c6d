#!/usr/bin/env bash
# tools/ab_runs.sh -- A/B of libolfx.so builds over several processes each (memory placement differs
# per process): for each of <runs> rounds, each lib in turn runs each workload's bench line
# (median of 5 regions of 40 steps).  Usage: bash tools/ab_runs.sh <runs> "<workloads>" <lib>...
# (lib paths relative to the repo root; "main" = ol_dsp_amd/libolfx.so; lib@VAR=value runs it under
# that environment variable)
set -u
mkdir -p gpurun_out
runs=$1; wls=$2; shift 2
for r in $(seq 1 "$runs"); do
  for lib in "$@"; do
    kv=OLFX_AB_NONE=1
    case $lib in *@*) kv=${lib#*@}; lib=${lib%%@*} ;; esac
    [ "$lib" = main ] && lib=ol_dsp_amd/libolfx.so
    for w in $wls; do
      env "$kv" OLFX_LIB=$PWD/$lib timeout -k 10 300 python bench.py --workload "$w" --also "" --steps 40 --warmup 5 --cpu-seconds 0 \
          --no-parity --full-json "" > gpurun_out/ab.log 2>&1 || { tail -n 20 gpurun_out/ab.log; exit 1; }
      python3 - "$w" "$lib $kv" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[1]:12s} {sys.argv[2]:36s} {r['kernel_ms']:.4f} ms  regions {d['reps']['kernel_ms']}")
PY
    done
  done
done
