#!/usr/bin/env bash
# tools/gpu_r2.sh -- one GPU-box session for round 2: GPU tests, smoke, the driver's default bench
# line (chorus + also{...}) and a rocprofv3 kernel-stats pass of the same command.
# Every GPU step has its own time limit; a crash/abort/timeout ends the script (no retries).
# Usage (repo root, via gpurun):  bash tools/gpu_r2.sh [tests|bench|prof|all] ...
set -u
out=gpurun_out
mkdir -p "$out"
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp

step() {   # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"; tail -n 4 "$out/$name.log"
    if [ $rc -ne 0 ]; then echo "!! $name failed (rc=$rc): stopping"; exit $rc; fi
}

for m in "${@:-all}"; do
  case $m in
    tests|all)
      step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
      step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
  esac
  case $m in
    bench|all)
      step bench_default 900 python bench.py ;;
  esac
  case $m in
    prof|all)
      step prof_default 900 rocprofv3 --kernel-trace --stats -d "$out/prof_default" -o run --output-format csv -- \
          python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0
      # keep the per-kernel summary only (the full trace is large and scratch)
      find "$out/prof_default" -name '*kernel_trace.csv' -delete ;;
  esac
done
echo "== done $(date +%T)"
