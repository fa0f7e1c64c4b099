#!/bin/bash
# Session tests (cell path) + C5s bench + kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_sessions_gpu.py > gpurun_out/r03f_sess.log 2>&1 || { tail -40 gpurun_out/r03f_sess.log; exit 1; }
tail -3 gpurun_out/r03f_sess.log
timeout -k 10 300 python bench.py --config c5s --steps 5 --warmup 1 --no-cpu-baseline --no-pcie --no-wire > gpurun_out/r03f_c5s.json 2> gpurun_out/r03f_c5s.log || { tail -20 gpurun_out/r03f_c5s.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r03f_c5s.json')); print('c5s', round(d['value']/1e9,2), d['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03f_prof -o run --output-format csv -- python3 $R/bench.py --config c5s --steps 5 --warmup 1 --no-cpu-baseline --no-pcie --no-wire > $R/gpurun_out/r03f_prof.log 2>&1 || { tail -20 $R/gpurun_out/r03f_prof.log; exit 1; }
python3 - <<'P'
import csv, glob
f = glob.glob('/root/repo/gpurun_out/r03f_prof/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r["Name"][:90], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3))
P
