#!/bin/bash
cd "${GRAFT_REPO_ROOT}"
export PYTHONUNBUFFERED=1
T="tests/test_gpu_parity.py::test_random_streams_vs_oracle"
mkdir -p gpurun_out
echo "== dbg"; (cd _ab_dbg && timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu "$T" > ../gpurun_out/dbg.log 2>&1); grep -E "BADREL|PWRITE" gpurun_out/dbg.log | head -20; grep -E "Error|passed|failed" gpurun_out/dbg.log | cut -c1-300 | tail -3
