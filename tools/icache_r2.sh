#!/usr/bin/env bash
# tools/icache_r2.sh -- instruction-cache counters (one rocprofv3 --pmc run per pass, kernel trace
# only) for the given bench workloads.  Any failure ends the script (no retries).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export PASSES="SQC_ICACHE_HITS;SQC_ICACHE_MISSES;SQ_IFETCH SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES"
for w in "$@"; do
  timeout -k 10 400 bash tools/pmc_profile.sh "$w" 10 || exit $?
done
echo "== icache done"
