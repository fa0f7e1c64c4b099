#!/bin/bash
# r03 evidence: bench lines of C3 / C5 / C5s / C4, and the per-dispatch trace + roofline recomputation of C4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for cfg in c3 c5 c5s; do
  w=1; [ $cfg = c3 ] && w=2
  timeout -k 10 400 python3 bench.py --config $cfg --steps 12 --warmup $w --no-pcie --no-wire > gpurun_out/r03_bench_$cfg.json 2> gpurun_out/r03_bench_$cfg.log || { tail -5 gpurun_out/r03_bench_$cfg.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03_bench_$cfg.json')); print('$cfg', round(d['value']/1e9,2), round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],4))"
done
TAG=c4 CFG=c4 BENCH_ARGS="--gpus 1 --steps 12 --warmup 2 --no-pcie --no-wire" bash tools/gpu_trace.sh || exit 1
