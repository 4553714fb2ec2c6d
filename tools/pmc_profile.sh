#!/usr/bin/env bash
# tools/pmc_profile.sh -- PMC counter passes for one bench workload (one rocprofv3 run per pass,
# --pmc only with --kernel-trace; never combined with sys/runtime traces).
# Usage: bash tools/pmc_profile.sh <workload> [steps] [extra bench args...]
set -u
wl=${1:-chorus}; steps=${2:-20}; shift 2 || true
out=gpurun_out/pmc_$wl
mkdir -p "$out"
export TMPDIR=/tmp
# the build these counters belong to: tools/pmc_traffic.py stamps its JSON with this hash and
# bench.py attaches a traffic file only to the libolfx.so it was recorded with
sha256sum ol_dsp_amd/libolfx.so | cut -d' ' -f1 > "$out/libolfx.sha256"
passes=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU"
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
)
if [ -n "${PASSES:-}" ]; then IFS=';' read -r -a passes <<< "$PASSES"; fi
k=${PASS_BASE:-0}
for p in "${passes[@]}"; do
  k=$((k+1))
  echo "== pass $k: $p"
  timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex "_block_|voice_mix|predelay" --pmc $p -d "$out/p$k" -o run --output-format csv -- \
      python3 bench.py --workload "$wl" --also "" --steps "$steps" --warmup 2 --cpu-seconds 0 "$@" > "$out/p$k.log" 2>&1
  rc=$?
  echo "   rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$out/p$k.log"; exit $rc; fi
done
echo "== done"
