#!/usr/bin/env bash
# tools/gpu_ab.sh -- GPU tests selected by -k, then an A/B timing of build/ab variants against the
# in-tree library.  Usage: bash tools/gpu_ab.sh "<pytest -k expr>" "<workloads>" <lib>...
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
k=$1; wls=$2; shift 2
if [ -n "$k" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "$k" \
      > gpurun_out/ab_pytest.log 2>&1
  rc=$?; tail -n 3 gpurun_out/ab_pytest.log; [ $rc -ne 0 ] && exit $rc
fi
bash tools/ab.sh "$wls" "$@"
