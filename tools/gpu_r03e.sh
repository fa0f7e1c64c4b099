#!/bin/bash
# r03: key dictionary (multi-column keys) tests + the heap / session suites after the changes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest --maxfail 10 -v --timeout 120 --timeout-method thread tests/test_keydict_gpu.py \
  tests/test_heap_snapshot_gpu.py tests/test_route_gpu.py tests/test_record_lists_gpu.py > gpurun_out/r03e_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/r03e_pytest.log | tail -15
exit $rc
