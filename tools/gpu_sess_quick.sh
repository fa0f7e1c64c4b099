#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_sessions_gpu.py > gpurun_out/sess_quick.log 2>&1; echo rc=$?
tail -3 gpurun_out/sess_quick.log
