#!/bin/bash
# r04: C5 / C3 with the combiner's window passes forced off / on (FWA_OPT_WINDOW_PASSES) against the adaptive default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for c in c5 c3; do
  for o in "" "--option window_passes=0" "--option window_passes=1"; do
    timeout -k 10 300 python -u bench.py --config $c --steps 12 --warmup 2 --no-cpu-baseline --no-pcie --no-wire $o \
      2>gpurun_out/r04mp.log > gpurun_out/r04mp_tmp.json || { tail -5 gpurun_out/r04mp.log; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r04mp_tmp.json')); print('$c', '$o', '%.4g'%d['value'], '%.3f'%d['ms_per_step'], {k: round(v/12,3) for k,v in d['ingest_split_ms'].items()}, 'replay', d['roofline']['replay_records'])"
  done
done
