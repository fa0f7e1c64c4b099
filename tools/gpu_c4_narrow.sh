#!/bin/bash
# r05: one-word record-list entries (int32 key | int32 BIGINT sum): parity incl. the full-size C4 digests, then C4 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_record_lists_gpu.py > gpurun_out/r05_sp_nw_tests.log 2>&1 || { tail -40 gpurun_out/r05_sp_nw_tests.log; exit 1; }
tail -1 gpurun_out/r05_sp_nw_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_full_size_digests_gpu.py -k c4 > gpurun_out/r05_sp_nw_digest.log 2>&1 || { tail -30 gpurun_out/r05_sp_nw_digest.log; exit 1; }
tail -1 gpurun_out/r05_sp_nw_digest.log
for rep in 1 2; do for v in 0 -1; do
  timeout -k 10 300 python -u bench.py --config c4 --option narrow_entries=$v > gpurun_out/r05_c4_nw$v.$rep.json 2> gpurun_out/r05_c4_nw$v.$rep.log || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r05_c4_nw$v.$rep.json').read().strip().splitlines()[-1]); s=d['ingest_split_ms']; n=d['steps']; print('narrow=$v rep$rep', round(d['value']/1e9,2), round(d['ms_per_step'],3), 'push %.3f fire %.3f' % (s['total']/n, d['roofline_fire']['ms_per_step']))"
done; done
