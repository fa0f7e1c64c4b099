#!/bin/bash
# whole GPU suite + smoke on the tree as it stands
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest --maxfail 20 -v --timeout 120 --timeout-method thread -m gpu tests \
  > gpurun_out/r04suite_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r04suite_pytest.log | tail -15
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04suite_smoke.log 2>&1 || { cat gpurun_out/r04suite_smoke.log; exit 1; }
tail -1 gpurun_out/r04suite_smoke.log
