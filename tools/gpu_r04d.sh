#!/bin/bash
# r04: window-pass parity fix check + DECIMAL + C3 clear-on-fire on the GPU
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for v in "0 i64 window_passes=1" "5 i64 window_passes=1" "3 i64"; do
  echo "== debug_parity $v"
  timeout -k 10 120 python -u tools/debug_parity.py $v > gpurun_out/dbg_parity.log 2>&1; rc=$?
  grep -E "MISMATCH|only GPU|no mismatch|Error" gpurun_out/dbg_parity.log | cut -c1-300
  if [ $rc -gt 1 ]; then echo "rc=$rc: stop"; exit $rc; fi
done
timeout -k 10 900 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_decimal_gpu.py tests/test_gpu_parity.py tests/test_sql_nulls_gpu.py tests/test_skew_gpu.py > gpurun_out/r04d_tests.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r04d_tests.log | tail -30
exit $rc
