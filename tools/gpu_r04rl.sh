#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_record_lists_gpu.py -k "owned_range" > gpurun_out/r04rl.log 2>&1; rc=$?
grep -E "^E |passed|failed|Error" gpurun_out/r04rl.log | head -20; exit $rc
