#!/bin/bash
# Whole GPU suite + smoke, then the per-dispatch trace of the driver's bench command (tools/gpu_trace.sh).
# TAG names the outputs (default full). SKIP_TESTS=1 runs only the trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-full}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest --maxfail 20 -v --timeout 120 --timeout-method thread -m gpu tests \
    > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_pytest.log | tail -15
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { cat gpurun_out/${TAG}_smoke.log; exit 1; }
  tail -2 gpurun_out/${TAG}_smoke.log
fi
TAG=$TAG bash tools/gpu_trace.sh
