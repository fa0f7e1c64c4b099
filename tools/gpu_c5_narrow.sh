#!/bin/bash
# r05: narrow entries for a DOUBLE beside a FLOAT column (NW = 2): parity, then C5 A/B (narrow_entries=0 vs default)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_narrow_gpu.py tests/test_gpu_parity.py tests/test_bench_shapes_gpu.py > gpurun_out/r05_nw2_tests.log 2>&1 || { tail -40 gpurun_out/r05_nw2_tests.log; exit 1; }
tail -1 gpurun_out/r05_nw2_tests.log
for rep in 1 2; do for v in 0 -1; do
  timeout -k 10 300 python -u bench.py --config c5 --option narrow_entries=$v > gpurun_out/r05_c5_nw$v.$rep.json 2> gpurun_out/r05_c5_nw$v.$rep.log || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r05_c5_nw$v.$rep.json').read().strip().splitlines()[-1]); s=d['ingest_split_ms']; n=d['steps']; print('narrow=$v rep$rep', round(d['value']/1e9,2), round(d['ms_per_step'],3), 'P %.3f A %.3f fire %.3f' % (s['partition']/n, s['combine']/n, d['roofline_fire']['ms_per_step']))"
done; done
