#!/usr/bin/env bash
# tools/traffic_check.sh -- HBM traffic passes (separate --pmc runs) for the bench workloads, plus
# the C++ operator parity test.  Any failure ends the script (no retries).
# Usage (repo root, via gpurun): bash tools/traffic_check.sh [workload...]
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
make -s -C tests/cpp || exit 1
timeout -k 10 300 python -m pytest tests/test_cpp_operators.py -m gpu -q -p no:cacheprovider \
    > gpurun_out/cpp_operators.log 2>&1
rc=$?; echo "cpp operators rc=$rc"; tail -n 3 gpurun_out/cpp_operators.log
[ $rc -ne 0 ] && exit $rc
export PASSES="FETCH_SIZE;WRITE_SIZE;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum;TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum;TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
for wl in "${@:-chorus dattorro}"; do
  for w in $wl; do
    bash tools/pmc_profile.sh "$w" 20 || exit $?
  done
done
echo "== traffic done"
