set -u
mkdir -p gpurun_out
for n in 8192 16384 32768 65536; do
  timeout -k 10 200 python bench.py --workload voice --also "" --instances $n --steps 60 --warmup 5 --cpu-seconds 0 > gpurun_out/vs.log 2>&1 || { tail -5 gpurun_out/vs.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/vs.log').read().strip().splitlines()[-1]);r=d['roofline'];print($n, r['kernel_ms'], d['value'])"
done
