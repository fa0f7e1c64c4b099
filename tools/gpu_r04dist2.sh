#!/bin/bash
# r04: isolate the N=2 raw-plan failure: C2 with raw records, C4 with partials, C4 raw with the histogram fusion off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 FWA_DIST_BACKEND=gloo
run() {
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --steps 2 --warmup 1 "$@" > gpurun_out/r04d2.json 2> gpurun_out/r04d2.log
  rc=$?
  echo "== $* rc=$rc"; grep -h "EngineError\|Error:" gpurun_out/r04d2.log | head -3
  [ $rc -eq 0 ] && python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/r04d2.json') if l.startswith('{')][-1]; print(d['value'], d['config'].get('exchange'))"
  return 0
}
run --config c2 --exchange raw
run --config c4 --exchange partials --keys 1000000
run --config c4 --exchange raw --keys 1000000
