#!/usr/bin/env bash
# tools/chain_ab_r2.sh -- chain parity tests, A/B against build/ab/*.so, optional extra passes.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "chain" > gpurun_out/pytest_chain.log 2>&1 || { tail -30 gpurun_out/pytest_chain.log; exit 1; }
tail -2 gpurun_out/pytest_chain.log
bash tools/ab.sh "${AB_WL:-chain chain_65536}" main ${AB_LIBS:-build/ab/chain_v1.so} || exit 1
if [ -n "${TRAFFIC:-}" ]; then
  bash tools/traffic_r2.sh chain > gpurun_out/traffic_chain.log 2>&1 || { tail gpurun_out/traffic_chain.log; exit 1; }
  echo traffic ok
fi
if [ -n "${ICACHE:-}" ]; then timeout -k 10 600 bash tools/icache_r2.sh chain > gpurun_out/icache.log 2>&1 || exit 1; echo icache ok; fi
