#!/usr/bin/env bash
# tools/traffic.sh -- HBM traffic passes (one rocprofv3 --pmc run per pass, kernel trace only)
# for the given bench workloads.  Any failure ends the script (no retries).
# Usage (repo root, via gpurun): bash tools/traffic.sh <workload>...
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export PASSES="FETCH_SIZE;WRITE_SIZE;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum;TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum;TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
for w in "$@"; do
  bash tools/pmc_profile.sh "$w" 10 || exit $?
done
echo "== traffic done"
