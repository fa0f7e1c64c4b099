#!/bin/bash
# r05: the combiner's window passes (FWA_OPT_WINDOW_PASSES forced on) with 4 entries per lane
# (flink_amd/libflink_amd_mp4.so, built with -DFWA_MP_IT=4) against the oracle: random streams + forced modes check
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cp flink_amd/libflink_amd_mp4.so flink_amd/libflink_amd.so || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "random_streams" --force-option window_passes=1 > gpurun_out/r05_mp4_parity.log 2>&1; rc=$?
tail -5 gpurun_out/r05_mp4_parity.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u tests/forced_modes_check.py > gpurun_out/r05_mp4_forced.log 2>&1; rc2=$?
tail -5 gpurun_out/r05_mp4_forced.log
exit $(( rc | rc2 ))
