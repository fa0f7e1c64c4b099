#!/bin/bash
# Narrow FLOAT-column entries (NW 3): tests, then C5 with FWA_NARROW 0 / 1 and FWA_NIT3 default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_narrow_gpu.py > gpurun_out/ab_n3_tests.log 2>&1 || { tail -30 gpurun_out/ab_n3_tests.log; exit 1; }
tail -1 gpurun_out/ab_n3_tests.log
for v in 0 1 0 1; do
  FWA_NARROW=$v timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 1 --no-pcie --no-wire --no-cpu-baseline > gpurun_out/ab_n3_$v.json 2> gpurun_out/ab_n3_$v.log || { tail -20 gpurun_out/ab_n3_$v.log; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ab_n3_$v.json')); s=d['ingest_split_ms']; print('c5 narrow $v', round(d['value']/1e9,2), round(d['ms_per_step'],4), 'P %.3f A %.3f' % (s['partition']/10, s['combine']/10))"
done
