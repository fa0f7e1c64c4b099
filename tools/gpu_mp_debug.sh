#!/bin/bash
# r05: diagnose the 4-entry window-pass combiner's duplicate rows (tools/debug_parity.py on random stream config 0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cp flink_amd/libflink_amd_mp4.so flink_amd/libflink_amd.so || exit 1
timeout -k 10 120 python -u tools/debug_parity.py 0 i64 window_passes=1 > gpurun_out/r05_mp4_debug.log 2>&1; echo rc=$?
tail -30 gpurun_out/r05_mp4_debug.log
