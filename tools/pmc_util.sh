#!/usr/bin/env bash
# tools/pmc_util.sh -- utilisation counters (issue mix, stalls, TA/TCP/L2) for bench workloads, one
# rocprofv3 --pmc pass per counter group (each within gfx950's per-block limits).
# Usage: bash tools/pmc_util.sh "<workloads>" [steps]   -> gpurun_out/util_<workload>/pN
set -u
wls=${1:-chorus}; steps=${2:-10}
export TMPDIR=/tmp
passes=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAIT_INST_LDS"
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
  "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE"
  "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCR_TCP_STALL_CYCLES_sum"
  "TCC_HIT_sum TCC_MISS_sum"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32 SQ_THREAD_CYCLES_VALU"
)
for wl in $wls; do
  out=gpurun_out/util_$wl
  mkdir -p "$out"
  k=0
  for p in "${passes[@]}"; do
    k=$((k+1))
    echo "== $wl pass $k: $p"
    timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "_block_|voice_mix" --pmc $p -d "$out/p$k" -o run --output-format csv -- \
        python3 bench.py --workload "$wl" --also "" --steps "$steps" --warmup 2 --cpu-seconds 0 > "$out/p$k.log" 2>&1
    rc=$?
    echo "   rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$out/p$k.log"; exit $rc; fi
  done
done
echo "== done"
