#!/bin/bash
# r04: record-list fire with the next entry prefetched: record-list GPU tests, C4 bench + per-dispatch trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_record_lists_gpu.py > gpurun_out/r04k_tests.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed|Error" gpurun_out/r04k_tests.log | tail -10
[ $rc -ne 0 ] && exit $rc
CFG=c4 TAG=r04_c4 bash tools/gpu_trace.sh || exit 1
python3 - <<'PY'
import csv, re
for r in csv.DictReader(open('gpurun_out/tr_r04_c4_kernel_stats.csv')):
    if float(r['AverageNs']) > 50000:
        print('%8.3f ms avg %5s  %s' % (float(r['AverageNs']) / 1e6, r['Calls'], re.sub(r'\(anonymous namespace\)::', '', r['Name'])[:80]))
PY
