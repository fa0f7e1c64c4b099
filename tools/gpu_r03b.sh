#!/bin/bash
# r03: heap-layout tests after the reader fix, then the C2 trace and a C5s bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest --maxfail 10 -v --timeout 120 --timeout-method thread tests/test_heap_snapshot_gpu.py \
  tests/test_record_lists_gpu.py > gpurun_out/r03b_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/r03b_pytest.log | tail -15
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
TAG=c2 bash tools/gpu_trace.sh || exit 1
timeout -k 10 300 python3 bench.py --config c5s --steps 10 --warmup 2 > gpurun_out/r03b_c5s.json 2> gpurun_out/r03b_c5s.log || { tail -5 gpurun_out/r03b_c5s.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03b_c5s.json')); print('c5s', d['value']/1e9, d['ms_per_step'], d['roofline']['frac'])"
