#!/usr/bin/env bash
# tools/save_profiles.sh -- copy the judged artifacts of a tools/gpu_check.sh run from gpurun_out/
# (scratch) into profiles/<round>/ (tracked): the bench JSON lines, the rocprofv3 kernel stats and
# the GPU pytest log.  Usage: bash tools/save_profiles.sh [round=r1] [tag=latest] [workloads...]
set -eu
rnd=${1:-r1}; tag=${2:-latest}; shift 2 || true
wls=${*:-chorus dattorro voice chain fxrack voice_moog voice_poly}
dst=profiles/$rnd
mkdir -p "$dst"
for w in $wls; do
  log=gpurun_out/bench_$w.log
  [ -f "$log" ] || continue
  line=$(grep '^{"metric"' "$log" | tail -n 1 || true)
  [ -n "$line" ] && printf '%s\n' "$line" > "$dst/bench_${w}_${tag}.json"
done
for w in $wls; do
  d=gpurun_out/prof_$w
  [ -d "$d" ] || continue
  f=$(ls "$d"/*kernel_stats.csv 2>/dev/null | head -n 1 || true)
  [ -n "$f" ] && cp "$f" "$dst/${w}_${tag}_kernel_stats.csv"
done
[ -f gpurun_out/pytest_gpu.log ] && cp gpurun_out/pytest_gpu.log "$dst/pytest_gpu_${tag}.log"
ls "$dst"
