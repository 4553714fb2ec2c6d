#!/usr/bin/env bash
# tools/ab.sh -- A/B timing of experimental builds of libolfx.so (OLFX_LIB) on the GPU box.
# Usage: bash tools/ab.sh "<workloads>" <lib> [<lib>...]   (lib paths relative to the repo root;
# "main" = ol_dsp_amd/libolfx.so).  Each run is a short bench; stops at the first failure.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
wls=$1; shift
for rep in 1 2; do
  for lib in "$@"; do
    [ "$lib" = main ] && lib=ol_dsp_amd/libolfx.so
    for w in $wls; do
      OLFX_LIB=$PWD/$lib timeout -k 10 300 python bench.py --workload "$w" --also "" --steps 60 --warmup 5 --cpu-seconds 0 --no-parity --full-json "" \
          > gpurun_out/ab.log 2>&1
      rc=$?; [ $rc -ne 0 ] && { tail -n 20 gpurun_out/ab.log; exit $rc; }
      python - "$w" "$lib" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[1]:10s} {sys.argv[2]:32s} {d['value']:.4e}/s  {r['kernel']} {r['kernel_ms']:.4f} ms  frac {r['frac']:.3f}")
PY
    done
  done
done
