#!/usr/bin/env bash
# tools/pmc_probe.sh -- tools/pmc_util.sh's counter passes over tools/bw_probe's chorus-shape kernels
# (32 and 16 instances per wave), one rocprofv3 --pmc run per pass -> gpurun_out/util_probe/pN.
# Summary: python tools/pmc_util_summary.py probe "chorus_shape<32u>" (and "<16u>").
set -u
export TMPDIR=/tmp
out=gpurun_out/util_probe
mkdir -p "$out"
passes=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAIT_INST_LDS"
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
  "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE"
  "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCR_TCP_STALL_CYCLES_sum"
  "TCC_HIT_sum TCC_MISS_sum"
)
k=0
for p in "${passes[@]}"; do
  k=$((k+1))
  echo "== probe pass $k: $p"
  timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "chorus_shape" --pmc $p -d "$out/p$k" -o run \
      --output-format csv -- tools/bw_probe > "$out/p$k.log" 2>&1
  rc=$?
  echo "   rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$out/p$k.log"; exit $rc; fi
done
echo "== done"
