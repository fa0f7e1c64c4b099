#!/bin/bash
# Bench line + rocprofv3 kernel stats for the secondary configs (C3, C4, C5, C5s); each step under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/cfg
for cfg in ${CFGS:-c3 c4 c5 c5s}; do
  W=1; [ $cfg = c3 ] && W=2
  timeout -k 10 300 python -u bench.py --config $cfg --warmup $W --no-cpu-baseline --no-pcie --no-wire > gpurun_out/cfg/bench_$cfg.log 2>&1 || { echo "bench $cfg failed"; tail -5 gpurun_out/cfg/bench_$cfg.log; exit 1; }
  grep '^{' gpurun_out/cfg/bench_$cfg.log > gpurun_out/cfg/bench_$cfg.json
  python3 -c "import json; d=json.load(open('gpurun_out/cfg/bench_$cfg.json')); print('$cfg', round(d['value']/1e9,2), 'G rec/s', round(d['ms_per_step'],3), 'ms/step frac', round(d['roofline']['frac'],4))"
  (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/cfg/prof_$cfg -o run --output-format csv -- python3 $R/bench.py --config $cfg --warmup $W --steps 4 --no-cpu-baseline --no-pcie --no-wire > $R/gpurun_out/cfg/prof_$cfg.log 2>&1) || { echo "prof $cfg failed"; exit 1; }
done
exit 0
