#!/bin/bash
# r04: N>1 rehearsal on one GPU -- two ranks sharing the card over gloo (the driver's 8-GPU runs use RCCL), for the
# partial-accumulator plan (C2) and the raw-record plan (C4, chosen automatically), plus C2 with raw records
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 FWA_DIST_BACKEND=gloo
for args in "--config c2" "--config c4" "--config c2 --exchange raw"; do
  tag=$(echo $args | tr -d ' -')
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --steps 3 --warmup 1 $args > gpurun_out/r04dist_$tag.json 2> gpurun_out/r04dist_$tag.log || { grep -h "Error" gpurun_out/r04dist_$tag.log | head -5; exit 1; }
  echo "== $args"; python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/r04dist_$tag.json') if l.startswith('{')][-1]; print(d['value'], d['n_gpus'], d['config'].get('exchange'), d['ms_per_step'])"
done
