#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
FWA_DEBUG_CELL=1 timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_sessions_gpu.py -k "overflow or table_session" > gpurun_out/dbg_cell.log 2>&1; echo rc=$?
grep -E "\[cell\]|PASS|FAIL" gpurun_out/dbg_cell.log | head -40
FWA_DEBUG_CELL=1 timeout -k 10 300 python bench.py --config c5s --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --no-wire > gpurun_out/dbg_c5s.json 2> gpurun_out/dbg_c5s.log; echo rc=$?
grep "\[cell\]" gpurun_out/dbg_c5s.log | head; cat gpurun_out/dbg_c5s.json | cut -c1-200
