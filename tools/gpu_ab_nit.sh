#!/bin/bash
# A/B: combine3 entries per lane and chunk on the narrow C2 path (FWA_NIT 4 / 6 / 8).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_narrow_gpu.py > gpurun_out/ab_nit_tests.log 2>&1 || { tail -20 gpurun_out/ab_nit_tests.log; exit 1; }
for it in 4 8 6 4 8; do
  FWA_NIT=$it timeout -k 10 300 python bench.py --steps 14 --warmup 1 --no-pcie --no-wire --no-cpu-baseline > gpurun_out/ab_nit$it.json 2> gpurun_out/ab_nit$it.log || { tail -20 gpurun_out/ab_nit$it.log; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ab_nit$it.json')); s=d['ingest_split_ms']; print('nit $it', round(d['value']/1e9,2), round(d['ms_per_step'],4), 'P %.3f A %.3f' % (s['partition']/14, s['combine']/14))"
done
