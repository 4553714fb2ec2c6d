#!/usr/bin/env bash
# tools/gpu_iter.sh -- one iteration on the GPU box: a subset of the GPU tests, then benches and
# (optionally) HBM-traffic passes for the given workloads.  Stops at the first failure.
# Usage: bash tools/gpu_iter.sh "<pytest -k expr>" "<bench workloads>" [traffic]
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
kexpr=${1:-}; wls=${2:-chorus}; traffic=${3:-}
if [ -n "$kexpr" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider -k "$kexpr" > gpurun_out/pytest_iter.log 2>&1
  rc=$?; tail -n 5 gpurun_out/pytest_iter.log; [ $rc -ne 0 ] && exit $rc
fi
for w in $wls; do
  timeout -k 10 300 python bench.py --workload "$w" --steps 60 --warmup 5 --cpu-seconds 0 > "gpurun_out/bench_$w.log" 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -n 20 "gpurun_out/bench_$w.log"; exit $rc; }
  python - "$w" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/bench_{sys.argv[1]}.log").read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[1]:10s} {d['value']:.4e} frames/s  kernel {r['kernel']} {r['kernel_ms']:.4f} ms  frac {r['frac']:.3f}")
PY
done
if [ -n "$traffic" ]; then
  export PASSES="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum;TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum;FETCH_SIZE;WRITE_SIZE"
  for w in $wls; do rm -rf "gpurun_out/pmc_$w"; bash tools/pmc_profile.sh "$w" 20 > /dev/null || exit $?; done
fi
echo "== iter done"
