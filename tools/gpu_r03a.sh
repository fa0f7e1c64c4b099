#!/bin/bash
# r03: parity of the changed areas (heap layout, nullable partials / snapshots), then the C2 trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_heap_snapshot_gpu.py \
  tests/test_sql_nulls_gpu.py tests/test_snapshot_gpu.py "tests/test_gpu_parity.py::test_shift_time_zone_sessions_vs_oracle" \
  "tests/test_gpu_parity.py::test_reference_kats_shift_time_zone_on_gpu" "tests/test_gpu_parity.py::test_two_phase_partials_vs_oracle" > gpurun_out/r03a_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error|error" gpurun_out/r03a_pytest.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_trace.sh
