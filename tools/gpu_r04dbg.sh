#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 \
  tools/debug_raw_c4b.py > gpurun_out/r04dbg.log 2>&1; rc=$?
grep -E "^rank|Error" gpurun_out/r04dbg.log | head -20; exit $rc
