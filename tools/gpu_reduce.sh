#!/bin/bash
# r05: DataStream built-in reductions on the GPU, then the parity suite for regressions
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_reduce_gpu.py \
  > gpurun_out/r05_reduce.log 2>&1; rc=$?; tail -25 gpurun_out/r05_reduce.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_narrow_gpu.py \
  > gpurun_out/r05_reduce_parity.log 2>&1; rc=$?; tail -3 gpurun_out/r05_reduce_parity.log; exit $rc
