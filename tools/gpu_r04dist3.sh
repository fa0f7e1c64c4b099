#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 FWA_DIST_BACKEND=gloo BENCH_DEBUG_KEYS=1
for b in 4194304; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 \
    bench.py --gpus 2 --steps 2 --warmup 1 --config c4 --exchange raw --batch $b > gpurun_out/r04d3.json 2> gpurun_out/r04d3_$b.log
  echo "== batch $b rc=$?"; grep -h "EngineError\|foreign" gpurun_out/r04d3_$b.log | head -12
done
exit 0
