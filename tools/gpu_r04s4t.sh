#!/bin/bash
# Session tests, a C5s bench and the s4 SQ pass on one box (the [cell][kid] LDS layout of s4_group).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_sessions_gpu.py > gpurun_out/r04s4t_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04s4t_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config c5s --steps 20 --warmup 3 --no-cpu-baseline --no-pcie --no-wire > gpurun_out/r04s4t_bench.json 2> gpurun_out/r04s4t_bench.err || exit $?
cat gpurun_out/r04s4t_bench.json
bash tools/gpu_sq_s4.sh
