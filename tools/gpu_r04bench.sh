#!/bin/bash
# r04 closing bench lines: the driver's default command (C2 with cpu_baseline / pcie / wire legs) and every other
# config at the driver's step counts, each under its own time limit; JSON lines to gpurun_out/r04_bench_<cfg>.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u bench.py > gpurun_out/r04_bench_c2.json 2> gpurun_out/r04_bench_c2.log || { tail -5 gpurun_out/r04_bench_c2.log; exit 1; }
echo "== c2"; python3 -c "import json; d=json.load(open('gpurun_out/r04_bench_c2.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'))"
for c in ${CONFIGS:-c3 c4 c5 c5s}; do
  W=5; [ $c = c3 ] && W=5
  timeout -k 10 400 python -u bench.py --config $c --gpus 1 --steps 20 --warmup $W > gpurun_out/r04_bench_$c.json 2> gpurun_out/r04_bench_$c.log || { tail -5 gpurun_out/r04_bench_$c.log; exit 1; }
  echo "== $c"; python3 -c "import json; d=json.load(open('gpurun_out/r04_bench_$c.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('traffic'))"
done
