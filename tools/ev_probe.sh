#!/usr/bin/env bash
# tools/ev_probe.sh -- note-event host path: control GPU tests, the voice / voice_events legs with the
# control-path trace, and per-step host times (tools/step_probe.py).  Stops at the first failure.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_control.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread -k "event or voice or control" > gpurun_out/ev_pytest.log 2>&1 || { tail -20 gpurun_out/ev_pytest.log; exit 1; }
tail -2 gpurun_out/ev_pytest.log
OLFX_TRACE_CONTROL=1 timeout -k 10 300 python bench.py --workload voice --also voice_events --steps 20 --warmup 5 --cpu-seconds 0 \
    > gpurun_out/ev_bench.log 2>&1 || { tail -20 gpurun_out/ev_bench.log; exit 1; }
grep -v '^{' gpurun_out/ev_bench.log | tail -8
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/ev_bench.log") if l.startswith('{"metric"')][-1])
print("voice", d["roofline"]["kernel_ms"], "events", d["also"]["voice_events"]["roofline"]["kernel_ms"], d["also"]["voice_events"]["control"])
PY
K=40 timeout -k 10 300 python tools/step_probe.py > gpurun_out/ev_steps.log 2>&1 || { tail -20 gpurun_out/ev_steps.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/ev_steps.log").read().strip().splitlines()[-1])
for k, v in d.items():
    print(k, {kk: vv for kk, vv in v.items() if kk != "host_us"})
PY
