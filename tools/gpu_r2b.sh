#!/usr/bin/env bash
# tools/gpu_r2b.sh -- one GPU-box session: every -m gpu test, the C++ operator binaries (their
# per-sample calls/s line), smoke, the driver's default bench line, a rocprofv3 kernel-stats pass
# of the same command, and HBM-traffic passes for the chain.  Each GPU step has its own time
# limit; a failure ends the script (no retries).
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
    echo "   rc=$rc"; tail -n 3 "$out/$name.log"
    if [ $rc -ne 0 ]; then echo "!! $name failed (rc=$rc): stopping"; exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread
step cpp_operators 300 tests/cpp/test_operators
step cpp_ref_surface 300 tests/cpp/test_ref_surface
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 900 python bench.py
step prof_default 900 rocprofv3 --kernel-trace --stats -d "$out/prof_default" -o run --output-format csv -- \
    python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0
find "$out/prof_default" -name '*kernel_trace.csv' -delete
if [ -n "${TRAFFIC:-}" ]; then
  step traffic 900 bash tools/traffic_r2.sh $TRAFFIC
fi
echo "== done $(date +%T)"
