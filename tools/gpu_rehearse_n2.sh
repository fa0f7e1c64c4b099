#!/bin/bash
# N=2 rehearsal of bench.py's multi-GPU path on one GPU: two ranks over gloo (FWA_DIST_BACKEND=gloo; RCCL refuses two
# ranks on one device), the two-phase plan (C2) and the raw-record plan (C4, reduce); logs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r06_n2}
port=29511
for cfg in ${CFGS:-c2 reduce c4}; do
  port=$((port+1))
  FWA_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --config $cfg --steps 4 --warmup 2 \
    > gpurun_out/${T}_$cfg.json 2> gpurun_out/${T}_$cfg.log || { tail -20 gpurun_out/${T}_$cfg.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/${T}_$cfg.json').read().strip().splitlines()[-1]); print('$cfg', d['n_gpus'], round(d['value']/1e9,2), 'G rec/s', d['config']['exchange'][:40], 'rows', d['rows_emitted'], 'dropped', d['late_dropped'])"
done
