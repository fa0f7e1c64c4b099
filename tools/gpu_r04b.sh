#!/bin/bash
# r04: whole GPU suite after the switch cleanup, then the batch-size sweep (MALL residency of the buckets) and the
# Phase P / A clock profile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest --maxfail 10 -q --timeout 120 --timeout-method thread -m gpu tests \
  > gpurun_out/r04b_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r04b_pytest.log | tail -15
[ $rc -gt 1 ] && exit $rc
BATCHES="2097152 4194304 8388608 16777216 67108864" RECS=536870912 bash tools/gpu_batchsweep.sh || exit 1
bash tools/gpu_pprof.sh
