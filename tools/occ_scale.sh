#!/usr/bin/env bash
# tools/occ_scale.sh -- kernel time vs instances per GPU for the given workloads (waves per SIMD
# follow the instance count).  Usage: bash tools/occ_scale.sh "<workloads>" "<instance counts>"
set -u
mkdir -p gpurun_out
for w in $1; do
  for n in $2; do
    timeout -k 10 200 python bench.py --workload $w --also "" --instances $n --steps 60 --warmup 5 --cpu-seconds 0 > gpurun_out/occ.log 2>&1 || { tail -5 gpurun_out/occ.log; exit 1; }
    python3 -c "
import json;d=json.loads(open('gpurun_out/occ.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$w', $n, round(r['kernel_ms'],4), '%.3e' % d['value'], round(r['frac'],3))"
  done
done
