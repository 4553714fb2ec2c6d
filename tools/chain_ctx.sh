#!/usr/bin/env bash
# tools/chain_ctx.sh -- the chain legs alone and in the bench's leg order, per library (GPU box).
# Usage: bash tools/chain_ctx.sh <lib>...   ("main" = ol_dsp_amd/libolfx.so)
set -u
mkdir -p gpurun_out
for lib in "$@"; do
  [ "$lib" = main ] && lib=ol_dsp_amd/libolfx.so
  for spec in "chain_65536:" "chain_rpd:chain_65536" "dattorro:chain_rpd,chain_65536"; do
    w=${spec%%:*}; also=${spec#*:}
    OLFX_LIB=$PWD/$lib timeout -k 10 300 python bench.py --workload "$w" --also "$also" --steps 20 --warmup 5 \
        --cpu-seconds 0 --no-parity --full-json "" > gpurun_out/ctx.log 2>&1 || { tail -n 20 gpurun_out/ctx.log; exit 1; }
    python - "$lib" "$w" "$also" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ctx.log").read().strip().splitlines()[-1])
legs = [(sys.argv[2], d["roofline"]["kernel_ms"])] + [(k, v["kernel_ms"]) for k, v in d.get("also", {}).items()]
print(f"{sys.argv[1]:28s} " + "  ".join(f"{k}={v:.4f}" for k, v in legs))
PY
  done
done
