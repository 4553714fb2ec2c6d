#!/usr/bin/env bash
# tools/save_traffic.sh -- summarise the PMC traffic passes merged from the GPU box
# (gpurun_out/pmc_<workload>, tools/traffic.sh) into profiles/traffic_<workload>.json, each
# stamped with the libolfx.so hash the counters were taken with (tools/pmc_profile.sh).
# Usage: bash tools/save_traffic.sh <workload>...
set -eu
for w in "$@"; do
  case $w in
    chain) n=16384 ;;
    *) n=65536 ;;
  esac
  python3 tools/pmc_traffic.py "$w" "$n" 256 "_block_" --out "profiles/traffic_$w.json" | tail -3
done
