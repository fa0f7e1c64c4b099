#!/bin/bash
# A/B: narrow entries as u64 + u16 slice (two streams) vs 12-byte {key, value, slice} (FWA_NARROW12=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
FWA_NARROW12=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_narrow_gpu.py > gpurun_out/ab_n12_tests.log 2>&1 || { tail -20 gpurun_out/ab_n12_tests.log; exit 1; }
tail -1 gpurun_out/ab_n12_tests.log
for v in 0 1 0 1; do
  FWA_NARROW12=$v timeout -k 10 300 python bench.py --steps 14 --warmup 1 --no-pcie --no-wire --no-cpu-baseline > gpurun_out/ab_n12_$v.json 2> gpurun_out/ab_n12_$v.log || { tail -20 gpurun_out/ab_n12_$v.log; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ab_n12_$v.json')); s=d['ingest_split_ms']; print('n12 $v', round(d['value']/1e9,2), round(d['ms_per_step'],4), 'P %.3f A %.3f' % (s['partition']/14, s['combine']/14))"
done
