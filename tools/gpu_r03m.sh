#!/bin/bash
# Record lists (sync-free scatter) + C4; narrow 8192-record tiles A/B on C2; slide fire + C3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_record_lists_gpu.py > gpurun_out/r03m_rl.log 2>&1 || { tail -30 gpurun_out/r03m_rl.log; exit 1; }
tail -1 gpurun_out/r03m_rl.log
FWA_NITEMS8=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_narrow_gpu.py > gpurun_out/r03m_narrow.log 2>&1 || { tail -30 gpurun_out/r03m_narrow.log; exit 1; }
tail -1 gpurun_out/r03m_narrow.log
timeout -k 10 400 python3 bench.py --config c4 --steps 12 --warmup 2 --no-pcie --no-wire > gpurun_out/r03m_c4.json 2> gpurun_out/r03m_c4.log || { tail -5 gpurun_out/r03m_c4.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03m_c4.json')); print('c4', round(d['value']/1e9,2), round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],4))"
for v in 0 1 0 1; do
  FWA_NITEMS8=$v timeout -k 10 300 python bench.py --steps 14 --warmup 1 --no-pcie --no-wire --no-cpu-baseline > gpurun_out/r03m_c2_i8_$v.json 2> gpurun_out/r03m_c2_i8_$v.log || { tail -20 gpurun_out/r03m_c2_i8_$v.log; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/r03m_c2_i8_$v.json')); s=d['ingest_split_ms']; print('c2 items8=$v', round(d['value']/1e9,2), round(d['ms_per_step'],4), 'P %.3f A %.3f' % (s['partition']/14, s['combine']/14))"
done
bash tools/gpu_c3.sh
