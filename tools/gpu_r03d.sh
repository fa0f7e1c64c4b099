#!/bin/bash
# r03: session segment kernel: session parity suites, heap tests, then a C5s kernel profile (and the r02 path for A/B).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest --maxfail 10 -v --timeout 120 --timeout-method thread tests/test_sessions_gpu.py \
  tests/test_heap_snapshot_gpu.py tests/test_late_firing_gpu.py tests/test_sql_nulls_gpu.py tests/test_bench_shapes_gpu.py \
  "tests/test_gpu_parity.py" > gpurun_out/r03d_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/r03d_pytest.log | tail -15
[ $rc -ne 0 ] && exit $rc
R=$PWD
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_c5s
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c5s -o run --output-format csv -- \
  python3 $R/bench.py --config c5s --steps 5 --warmup 1 > $R/gpurun_out/r03d_c5s.json 2> $R/gpurun_out/r03d_c5s.log || { tail -5 $R/gpurun_out/r03d_c5s.log; exit 1; }
cd $R
f=$(find gpurun_out/prof_c5s -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r03d_c5s_kernel_stats.csv
python3 - <<'PY'
import csv, json
rows = list(csv.reader(open('gpurun_out/r03d_c5s_kernel_stats.csv')))
for r in rows[1:16]:
    print(r[0][:70].ljust(70), r[1], "%.3f" % (float(r[2]) / 1e6), "%.3f" % (float(r[3]) / 1e6))
d = json.load(open('gpurun_out/r03d_c5s.json')); print('c5s (profiled)', d['value'] / 1e9, d['ms_per_step'])
PY
timeout -k 10 300 python3 bench.py --config c5s --steps 10 --warmup 2 > gpurun_out/r03d_c5s_bench.json 2> gpurun_out/r03d_c5s_bench.log || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r03d_c5s_bench.json')); print('c5s', d['value']/1e9, d['ms_per_step'], d['roofline']['frac'])"
FWA_SESS_SCAN=1 timeout -k 10 300 python3 bench.py --config c5s --steps 10 --warmup 2 > gpurun_out/r03d_c5s_scan.json 2> gpurun_out/r03d_c5s_scan.log || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r03d_c5s_scan.json')); print('c5s r02 path', d['value']/1e9, d['ms_per_step'])"
