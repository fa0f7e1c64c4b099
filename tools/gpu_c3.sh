#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "slide or c3 or random_streams" > gpurun_out/c3_tests.log 2>&1 || { tail -30 gpurun_out/c3_tests.log; exit 1; }
tail -1 gpurun_out/c3_tests.log
timeout -k 10 400 python3 bench.py --config c3 --steps 12 --warmup 2 --no-pcie --no-wire > gpurun_out/r03_bench_c3.json 2> gpurun_out/r03_bench_c3.log || { tail -5 gpurun_out/r03_bench_c3.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03_bench_c3.json')); print('c3', round(d['value']/1e9,2), round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],4), 'fire ms/step %.3f' % (d['fire']['ms']/12))"
