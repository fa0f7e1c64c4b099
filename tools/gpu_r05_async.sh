#!/bin/bash
# r05: the fire stream (asynchronous TUMBLE fire beside the next push): parity, then C2 bench sync vs async, and a
# kernel trace of the async loop
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_async_watermark_gpu.py tests/test_gpu_parity.py \
  > gpurun_out/r05_async_tests.log 2>&1 || { tail -30 gpurun_out/r05_async_tests.log; exit 1; }
tail -2 gpurun_out/r05_async_tests.log
for mode in nofresh sync async; do
  extra=""; [ $mode = async ] && extra="--async-fire"; [ $mode = nofresh ] && extra="--option ingest_variant=1"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie --no-wire $extra > gpurun_out/r05_c2_$mode.json 2> gpurun_out/r05_c2_$mode.log || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r05_c2_$mode.json').read().strip().splitlines()[-1]); print('$mode', d['value']/1e9, d['ms_per_step'])"
done
TAG=r05_c2_async2 BENCH_ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-pcie --no-wire --async-fire" bash tools/gpu_trace.sh || exit 1
python3 tools/trace_gaps.py gpurun_out/tr_r05_c2_async2_kernel_trace.csv 40 | tail -30
