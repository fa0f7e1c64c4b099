#!/bin/bash
# Narrow-entry tests, the parity suite, and the C2 bench (narrow vs 64-bit entries).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_narrow_gpu.py tests/test_gpu_parity.py tests/test_sessions_gpu.py > gpurun_out/r03g_tests.log 2>&1 || { tail -30 gpurun_out/r03g_tests.log; exit 1; }
tail -2 gpurun_out/r03g_tests.log
for v in 1 0; do
  FWA_NARROW=$v timeout -k 10 300 python bench.py --steps 14 --warmup 1 --no-pcie --no-wire --no-cpu-baseline > gpurun_out/r03g_c2_n$v.json 2> gpurun_out/r03g_c2_n$v.log || { tail -20 gpurun_out/r03g_c2_n$v.log; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/r03g_c2_n$v.json')); print('c2 narrow=$v', round(d['value']/1e9,2), d['ms_per_step'], round(d['roofline']['frac'],4), d['ingest_split_ms'])"
done
