#!/usr/bin/env bash
# tools/gpu_r6.sh -- GPU-box steps for round 6.  Every GPU step has its own time limit; a crash,
# abort or timeout ends the script (no retries).
# Usage (repo root, via gpurun):  bash tools/gpu_r6.sh <mode>...
#   t:<pytest -k expr>   GPU tests matching the expression
#   tests                every GPU test, then smoke()
#   b:<workload>         one workload's bench line (20 steps, no CPU baseline)
#   p:<workload>         rocprofv3 kernel stats of that bench line (-> gpurun_out/prof_<w>)
#   tr:<workload>        HBM traffic passes (tools/traffic.sh)
#   bench                the driver's default line
#   tl:<lib>:<k>         GPU tests matching <k> against an experimental build (OLFX_LIB=<lib>)
#   te:<VAR=v>:<k>       GPU tests matching <k> with the environment variable VAR=v
#   ts:<k>               GPU tests matching <k>, with their printed output (-s)
#   abe:<workload>:<VAR=v> A/B: the workload under the default and VAR=v, three times each
#   abm:<w1,w2>:<lib1,lib2> A/B of the main build against several libs over several workloads
#   util:<workload>      utilisation counter passes (tools/pmc_util.sh)
#   abl:<workload>:<lib> A/B of the main build against <lib> (tools/ab.sh)
#   occ:<workloads>:<ns> kernel time against instances (tools/occ_scale.sh), e.g. occ:dattorro,chain:16384,65536
#   occe:<VAR=v>:<workloads>:<ns>  the same under an environment variable
#   probe                tools/bw_probe (built here: hipcc ... -o tools/bw_probe), then the chorus's
#                        bench line, on the same box
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

for m in "$@"; do
  case $m in
    t:*)
      k=${m#t:}
      step "pytest_$(echo "$k" | tr -c 'a-zA-Z0-9_' '_')" 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider \
          --timeout 120 --timeout-method thread -k "$k" ;;
    tl:*)
      r=${m#tl:}; lib=${r%%:*}; k=${r#*:}
      step "pytest_lib_$(echo "$k" | tr -c 'a-zA-Z0-9_' '_')" 600 env OLFX_LIB=$PWD/$lib python -u -m pytest tests -m gpu -x -v \
          -p no:cacheprovider --timeout 120 --timeout-method thread -k "$k" ;;
    te:*)
      r=${m#te:}; kv=${r%%:*}; k=${r#*:}
      step "pytest_env_$(echo "$kv$k" | tr -c 'a-zA-Z0-9_' '_')" 600 env "$kv" python -u -m pytest tests -m gpu -x -v \
          -p no:cacheprovider --timeout 120 --timeout-method thread -k "$k" ;;
    ts:*)
      k=${m#ts:}
      step "pytest_s_$(echo "$k" | tr -c 'a-zA-Z0-9_' '_')" 600 python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider \
          --timeout 120 --timeout-method thread -k "$k"
      grep -E "rel err|PASSED|FAILED" "$out/pytest_s_$(echo "$k" | tr -c 'a-zA-Z0-9_' '_').log" ;;
    abl:*)
      r=${m#abl:}; w=${r%%:*}; lib=${r#*:}
      step "abl_$w" 600 bash tools/ab.sh "$w" main "$lib"
      cat "$out/abl_$w.log" ;;
    abm:*)
      r=${m#abm:}; w=${r%%:*}; libs=${r#*:}
      step "abm_$(echo "$w" | tr -c 'a-zA-Z0-9_' '_')" 900 bash tools/ab.sh "${w//,/ }" main ${libs//,/ }
      cat "$out/abm_$(echo "$w" | tr -c 'a-zA-Z0-9_' '_').log" ;;
    tests)
      step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
      step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    b:*)
      w=${m#b:}
      step "bench_$w" 300 python bench.py --workload "$w" --also "" --steps 20 --warmup 5 --cpu-seconds 0 --full-json "" ;;
    p:*)
      w=${m#p:}; wl=$w; [ "$w" = chain_16384 ] && wl=chain
      step "prof_$w" 300 rocprofv3 --kernel-trace --stats -d "$out/prof_$w" -o run --output-format csv -- \
          python3 bench.py --workload "$wl" --also "" --steps 20 --warmup 5 --cpu-seconds 0 --no-parity --full-json ""
      find "$out/prof_$w" -name '*kernel_trace.csv' -delete ;;
    tr:*)
      w=${m#tr:}
      step "traffic_$w" 600 bash tools/traffic.sh "$w" ;;
    abe:*)
      r=${m#abe:}; w=${r%%:*}; kv=${r#*:}
      for r in 1 2 3; do
        step "abe_${w}_default_$r" 300 python bench.py --workload "$w" --also "" --steps 50 --warmup 5 \
            --cpu-seconds 0 --no-parity --full-json ""
        step "abe_${w}_env_$r" 300 env "$kv" python bench.py --workload "$w" --also "" --steps 50 --warmup 5 --cpu-seconds 0 \
            --no-parity --full-json ""
      done ;;
    bench)
      step bench_default 900 python bench.py --steps 20 --warmup 5 ;;
    util:*)
      w=${m#util:}
      step "util_$w" 900 bash tools/pmc_util.sh "$w" 10 ;;
    occ:*)
      r=${m#occ:}; w=${r%%:*}; ns=${r#*:}
      step "occ_$(echo "$w$ns" | tr -c 'a-zA-Z0-9_' '_')" 600 bash tools/occ_scale.sh "${w//,/ }" "${ns//,/ }"
      cat "$out/occ_$(echo "$w$ns" | tr -c 'a-zA-Z0-9_' '_').log" ;;
    occe:*)
      r=${m#occe:}; kv=${r%%:*}; r=${r#*:}; w=${r%%:*}; ns=${r#*:}
      step "occe_$(echo "$kv$w$ns" | tr -c 'a-zA-Z0-9_' '_')" 600 env "$kv" bash tools/occ_scale.sh "${w//,/ }" "${ns//,/ }"
      cat "$out/occe_$(echo "$kv$w$ns" | tr -c 'a-zA-Z0-9_' '_').log" ;;
    probe)
      step bw_probe 300 tools/bw_probe
      cat "$out/bw_probe.log"
      step bench_chorus_probe 300 python bench.py --workload chorus --also "" --steps 20 --cpu-seconds 0 --no-parity \
          --full-json ""
      cat "$out/bench_chorus_probe.log" ;;
    *) echo "unknown mode $m"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
