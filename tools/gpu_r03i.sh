#!/bin/bash
# Skew tests + smoke + C2 trace (the rest of the suite passed in r03h).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_skew_gpu.py > gpurun_out/r03i_skew.log 2>&1 || { tail -20 gpurun_out/r03i_skew.log; exit 1; }
tail -1 gpurun_out/r03i_skew.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03i_smoke.log 2>&1 || { cat gpurun_out/r03i_smoke.log; exit 1; }
tail -1 gpurun_out/r03i_smoke.log
SKIP_TESTS=1 TAG=r03i bash tools/gpu_full.sh
