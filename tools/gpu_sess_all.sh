#!/bin/bash
# Every GPU test file that exercises the session paths.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_sessions_gpu.py tests/test_gpu_parity.py tests/test_heap_snapshot_gpu.py tests/test_snapshot_gpu.py tests/test_sql_nulls_gpu.py > gpurun_out/sess_all.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/sess_all.log | tail -8
exit $rc
