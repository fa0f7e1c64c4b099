#!/bin/bash
# Parity suites that fire multi-accumulator TUMBLE windows, then C5 with fire_multi_kernel (variant 0) against the
# generic fire (variant 32).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r06_fm}
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_decimal_gpu.py tests/test_snapshot_gpu.py tests/test_narrow_gpu.py \
  > gpurun_out/${T}_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
for v in 0 32 0 32; do
  timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --option ingest_variant=$v > gpurun_out/${T}_v$v.json \
    2> gpurun_out/${T}_v$v.log || { tail -5 gpurun_out/${T}_v$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/${T}_v$v.json').read().strip().splitlines()[-1]); print('v$v', round(d['value']/1e9,2), round(d['ms_per_step'],3), 'fire', round(d['roofline_fire']['ms_per_step'],3))"
done
