#!/bin/bash
# Flat layout: skew tests and the bench A/B only (the parity suites passed in gpu_flat.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_skew_gpu.py > gpurun_out/flat2_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/flat2_pytest.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
sed -n '/^for cfg/,$p' tools/gpu_flat.sh > /tmp/flat_bench.sh && bash /tmp/flat_bench.sh
