set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for also in "voice" "dattorro,chain_65536,chain,voice" "voice_moog,fxrack,voice"; do
  echo "== also=$also"
  OLFX_TRACE_CONTROL=1 timeout -k 10 300 python bench.py --workload chorus --also "$also" --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/probe.log 2>&1 || { tail -20 gpurun_out/probe.log; exit 1; }
  grep -i "trace\|control" gpurun_out/probe.log | grep -v '^{' | tail -6
  python3 - <<'PY'
import json
d=json.loads([l for l in open('gpurun_out/probe.log') if l.startswith('{')][0])
for k,v in d['also'].items(): print(k, round(v['ms_per_step'],4), round(v['roofline']['kernel_ms'],4))
PY
done
