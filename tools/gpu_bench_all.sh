#!/bin/bash
# Bench lines of every config (C2 with its CPU / PCIe / 64-bit-key / wire legs), each under its own limit; JSON lines
# in gpurun_out/<TAG>_bench_<cfg>.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r05}
for cfg in ${CFGS:-c2 c3 c4 c5 c5s}; do
  extra=""
  timeout -k 10 420 python -u bench.py --config $cfg $extra > gpurun_out/${T}_bench_$cfg.json 2> gpurun_out/${T}_bench_$cfg.log || { tail -5 gpurun_out/${T}_bench_$cfg.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/${T}_bench_$cfg.json').read().strip().splitlines()[-1]); print('$cfg', round(d['value']/1e9,2), 'G rec/s', round(d['ms_per_step'],3), 'ms/step, frac', round(d['roofline']['frac'],4), 'wide' if 'wide_keys' not in d else round(d['wide_keys']['value']/1e9,2))"
done
