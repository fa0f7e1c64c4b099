#!/bin/bash
# r03: heap layouts (DataStream SLIDE, Table SESSION added), then a C5s kernel profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest --maxfail 10 -v --timeout 120 --timeout-method thread tests/test_heap_snapshot_gpu.py \
  tests/test_snapshot_gpu.py tests/test_sessions_gpu.py > gpurun_out/r03c_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/r03c_pytest.log | tail -15
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
R=$PWD
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_c5s
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c5s -o run --output-format csv -- \
  python3 $R/bench.py --config c5s --steps 5 --warmup 1 > $R/gpurun_out/r03c_c5s.json 2> $R/gpurun_out/r03c_c5s.log || { tail -5 $R/gpurun_out/r03c_c5s.log; exit 1; }
cd $R
f=$(find gpurun_out/prof_c5s -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r03c_c5s_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.reader(open('gpurun_out/r03c_c5s_kernel_stats.csv')))
for r in rows[1:]:
    print(r[0][:70].ljust(70), r[1], "%.3f" % (float(r[2]) / 1e6), "%.3f" % (float(r[3]) / 1e6))
PY
