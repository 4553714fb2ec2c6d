#!/usr/bin/env bash
# tools/gpu_r3.sh -- GPU-box steps (rounds 3-4).  Every GPU step has its own time limit; a crash,
# abort or timeout ends the script (no retries).
# Usage (repo root, via gpurun):  bash tools/gpu_r3.sh <mode>...
#   ctl_tests  the control-path / tiling GPU tests (tests/test_gpu_control.py)
#   tests      every GPU test, then smoke()
#   ctl_bench  bench legs voice, voice_events, chain, chain_cc (20 steps, as the driver)
#   bench      the driver's default line (python bench.py)
#   prof       rocprofv3 kernel stats of the default line
#   prof_ctl   rocprofv3 kernel stats of the voice / chain legs, one CSV per workload
#   wl:<name>  one workload's bench line, kernel stats and HBM traffic passes
#   final      default bench line + kernel stats of it and of every workload (one CSV each)
#   util       utilisation counter passes (UTIL_WLS, default chorus fxrack voice chain chain_65536)
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

prof() {   # prof <name> <seconds> <bench args...>: kernel stats only (the full trace is scratch)
    local name=$1 secs=$2; shift 2
    step "prof_$name" "$secs" rocprofv3 --kernel-trace --stats -d "$out/prof_$name" -o run --output-format csv -- \
        python3 bench.py "$@"
    find "$out/prof_$name" -name '*kernel_trace.csv' -delete
}

for m in "$@"; do
  case $m in
    ctl_tests)
      step pytest_ctl 600 python -u -m pytest tests/test_gpu_control.py -m gpu -x -v -p no:cacheprovider \
          --timeout 300 --timeout-method thread ;;
    tests)
      step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
      step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    ctl_bench)
      step bench_ctl 600 python bench.py --steps 20 --warmup 5 --workload voice --also voice_events,chain,chain_cc \
          --cpu-seconds 0 ;;
    ctl_ab)   # control-packet delivery A/B: OLFX_COPY_BYTES=0 copies every packet through the big
              # slots, the default (64 KiB) reads small packets zero-copy from pinned host slots
      for cb in ${COPY_BYTES_AB:-0 65536}; do
        step "pytest_ctl_cb$cb" 600 env OLFX_COPY_BYTES=$cb python -u -m pytest tests/test_gpu_control.py -m gpu -x -q \
            -p no:cacheprovider --timeout 300 --timeout-method thread -k "not tiled"
        step "bench_ctl_cb$cb" 600 env OLFX_COPY_BYTES=$cb OLFX_TRACE_CONTROL=1 python bench.py --steps 20 --warmup 5 \
            --workload voice --also voice_events,chain,chain_cc --cpu-seconds 0 --no-parity
        for w in voice_events chain_cc; do
          step "prof_${w}_cb$cb" 300 env OLFX_COPY_BYTES=$cb rocprofv3 --kernel-trace --stats -d "$out/prof_${w}_cb$cb" \
              -o run --output-format csv -- python3 bench.py --workload $w --also "" --steps 20 --warmup 5 --cpu-seconds 0 --no-parity
          find "$out/prof_${w}_cb$cb" -name '*kernel_trace.csv' -delete
        done
      done ;;
    timeline)   # runtime-API + kernel timeline of the control legs (no counters)
      for w in voice_events voice; do
        step "tl_$w" 300 rocprofv3 --kernel-trace --hip-trace -d "$out/tl_$w" -o run --output-format csv -- \
            python3 bench.py --workload $w --also "" --steps 40 --warmup 5 --cpu-seconds 0
        python3 tools/timeline.py "$out/tl_$w" voice_block > "$out/tl_$w.txt" 2>&1
        find "$out/tl_$w" -name '*.csv' -delete
      done ;;
    bench)
      step bench_default 900 python bench.py --steps 20 --warmup 5 ;;
    prof)
      prof default 900 --steps 50 --warmup 5 --cpu-seconds 0 ;;
    prof_ctl)
      for w in voice voice_events chain chain_cc chain_65536; do
        prof "$w" 300 --workload "$w" --also "" --steps 20 --warmup 5 --cpu-seconds 0
      done ;;
    final)     # the round's artifacts: default bench line, its kernel stats, per-workload stats
      step bench_default 900 python bench.py --steps 20 --warmup 5
      prof default 900 --steps 50 --warmup 5 --cpu-seconds 0
      for w in chorus pitchshift dattorro chain chain_65536 voice voice_moog voice_events chain_cc fxrack; do
        prof "$w" 300 --workload "$w" --also "" --steps 20 --warmup 5 --cpu-seconds 0
      done ;;
    util)      # utilisation counters (tools/pmc_util.sh) of the VERDICT's kernels
      step util 900 bash tools/pmc_util.sh "${UTIL_WLS:-chorus fxrack voice chain chain_65536}" 10 ;;
    wl:*)      # one workload: bench line, kernel stats, HBM traffic passes (tools/traffic_r2.sh)
      w=${m#wl:}
      step "bench_$w" 300 python bench.py --workload "$w" --also "" --steps 20 --warmup 5 --cpu-seconds 0
      prof "$w" 300 --workload "$w" --also "" --steps 20 --warmup 5 --cpu-seconds 0
      step "traffic_$w" 600 bash tools/traffic_r2.sh "$w" ;;
    *) echo "unknown mode $m"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
