#!/bin/bash
# r04 closing validation: whole GPU suite + smoke on the final tree, then the C4 per-dispatch trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest --maxfail 20 -v --timeout 120 --timeout-method thread -m gpu tests \
  > gpurun_out/r04final_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r04final_pytest.log | tail -15
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04final_smoke.log 2>&1 || { cat gpurun_out/r04final_smoke.log; exit 1; }
tail -1 gpurun_out/r04final_smoke.log
CFG=c4 TAG=r04_c4 bash tools/gpu_trace.sh || exit 1
python3 - <<'PY'
import csv, re
for r in csv.DictReader(open('gpurun_out/tr_r04_c4_kernel_stats.csv')):
    if float(r['AverageNs']) > 50000:
        print('%8.3f ms avg %5s  %s' % (float(r['AverageNs']) / 1e6, r['Calls'], re.sub(r'\(anonymous namespace\)::', '', r['Name'])[:80]))
PY
