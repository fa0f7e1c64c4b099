#!/bin/bash
# Session (cell pre-aggregation) tests, then C5s with the s5 hash route (variant 0) against the s4 probe route (8).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r06_s5}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_sessions_gpu.py \
  tests/test_snapshot_prehashed_gpu.py tests/test_heap_snapshot_gpu.py > gpurun_out/${T}_sess.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_sess.log; [ $rc -ne 0 ] && exit $rc
for v in ${VARIANTS:-0 8 0 8}; do
  timeout -k 10 300 python bench.py --config c5s --no-cpu-baseline --option ingest_variant=$v > gpurun_out/${T}_v$v.json \
    2> gpurun_out/${T}_v$v.log || { tail -5 gpurun_out/${T}_v$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/${T}_v$v.json').read().strip().splitlines()[-1]); print('v$v', round(d['value']/1e9,2), round(d['ms_per_step'],3), round(d['ingest_split_ms']['total']/d['steps'],3))"
done
