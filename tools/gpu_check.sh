#!/usr/bin/env bash
# tools/gpu_check.sh -- one GPU-box session: tests, smoke, short benches (+ optional rocprof).
# Every GPU step has its own time limit; any crash/abort/timeout ends the script (no retries).
# Usage (from the repo root, via gpurun):  bash tools/gpu_check.sh [quick|full|prof]
set -u
mode=${1:-quick}
out=gpurun_out
mkdir -p "$out"
export PYTHONUNBUFFERED=1

step() {   # step <name> <seconds> <cmd...>; returns the command's status, stops on crash
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"; tail -n 3 "$out/$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; then
        echo "!! $name crashed or timed out (rc=$rc): stopping"; exit $rc
    fi
    return $rc
}

step pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench_chorus 400 python bench.py --steps 100 --warmup 10 --cpu-seconds 5
step bench_dattorro 400 python bench.py --workload dattorro --steps 40 --warmup 5 --cpu-seconds 5
if [ "$mode" = full ] || [ "$mode" = prof ]; then
    step bench_voice 300 python bench.py --workload voice --steps 100 --warmup 10 --cpu-seconds 3
    step bench_chain 400 python bench.py --workload chain --steps 40 --warmup 5 --cpu-seconds 3
    step bench_fxrack 400 python bench.py --workload fxrack --steps 60 --warmup 5 --cpu-seconds 3
    step bench_voice_moog 300 python bench.py --workload voice_moog --steps 60 --warmup 5 --cpu-seconds 3
    step bench_voice_poly 300 python bench.py --workload voice_poly --steps 100 --warmup 10 --cpu-seconds 0
fi
if [ "$mode" = prof ]; then
    export TMPDIR=/tmp
    step prof_chorus 600 rocprofv3 --kernel-trace --stats -d "$out/prof_chorus" -o run --output-format csv -- \
        python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0
    step prof_dattorro 600 rocprofv3 --kernel-trace --stats -d "$out/prof_dattorro" -o run --output-format csv -- \
        python3 bench.py --workload dattorro --steps 20 --warmup 3 --cpu-seconds 0
    step prof_voice 600 rocprofv3 --kernel-trace --stats -d "$out/prof_voice" -o run --output-format csv -- \
        python3 bench.py --workload voice --steps 50 --warmup 3 --cpu-seconds 0
    step prof_chain 600 rocprofv3 --kernel-trace --stats -d "$out/prof_chain" -o run --output-format csv -- \
        python3 bench.py --workload chain --steps 20 --warmup 3 --cpu-seconds 0
    step prof_fxrack 600 rocprofv3 --kernel-trace --stats -d "$out/prof_fxrack" -o run --output-format csv -- \
        python3 bench.py --workload fxrack --steps 30 --warmup 3 --cpu-seconds 0
    step prof_voice_moog 600 rocprofv3 --kernel-trace --stats -d "$out/prof_voice_moog" -o run --output-format csv -- \
        python3 bench.py --workload voice_moog --steps 30 --warmup 3 --cpu-seconds 0
    step prof_voice_poly 600 rocprofv3 --kernel-trace --stats -d "$out/prof_voice_poly" -o run --output-format csv -- \
        python3 bench.py --workload voice_poly --steps 50 --warmup 3 --cpu-seconds 0
fi
echo "== done $(date +%T)"
