#!/bin/bash
# Record-list tests + C4 bench; slide tests + C3 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_record_lists_gpu.py > gpurun_out/r03l_rl.log 2>&1 || { tail -30 gpurun_out/r03l_rl.log; exit 1; }
tail -1 gpurun_out/r03l_rl.log
timeout -k 10 400 python3 bench.py --config c4 --steps 12 --warmup 2 --no-pcie --no-wire > gpurun_out/r03l_c4.json 2> gpurun_out/r03l_c4.log || { tail -5 gpurun_out/r03l_c4.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03l_c4.json')); print('c4', round(d['value']/1e9,2), round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],4))"
bash tools/gpu_c3.sh
