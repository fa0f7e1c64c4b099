#!/bin/bash
# Parity suites touching the speculative fire and slot retirement, then the C2 trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_narrow_gpu.py tests/test_snapshot_gpu.py > gpurun_out/r03k_tests.log 2>&1 || { tail -30 gpurun_out/r03k_tests.log; exit 1; }
tail -1 gpurun_out/r03k_tests.log
SKIP_TESTS=1 TAG=r03k bash tools/gpu_full.sh > gpurun_out/r03k_trace.log 2>&1 || { tail -20 gpurun_out/r03k_trace.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/tr_r03k_roofline.json')); r=json.load(open('gpurun_out/tr_r03k.json')); print(round(r['value']/1e9,2), r['ms_per_step'], d['dominant']['frac'], d['step'])"
for ab in 0 1; do
  FWA_FSABL=$ab timeout -k 10 300 python3 bench.py --config c3 --steps 6 --warmup 2 --no-pcie --no-wire --no-cpu-baseline > gpurun_out/r03k_c3_fsabl$ab.json 2> gpurun_out/r03k_c3_fsabl$ab.log || { tail -5 gpurun_out/r03k_c3_fsabl$ab.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r03k_c3_fsabl$ab.json')); print('c3 fsabl $ab', round(d['value']/1e9,2), round(d['ms_per_step'],3), 'fire ms/step %.3f' % (d['fire']['ms']/6))"
done
