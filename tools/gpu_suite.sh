#!/bin/bash
# Whole GPU suite (full-size digest tests with their own longer limit), then smoke(). Logs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${TAG:-r05}
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_full_size_digests_gpu.py \
  > gpurun_out/${T}_digests.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_digests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 1000 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests --deselect tests/test_full_size_digests_gpu.py \
  > gpurun_out/${T}_gputest.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_gputest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
