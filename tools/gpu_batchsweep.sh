#!/bin/bash
# bench at several batch sizes (one process each): per-record kernel cost vs batch size
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for b in ${BATCHES:-4194304 16777216 67108864}; do
  steps=$(( ${RECS:-402653184} / b ))
  timeout -k 10 300 python -u bench.py --batch $b --steps $steps --warmup 2 --no-cpu-baseline > gpurun_out/bs_$b.json 2> gpurun_out/bs_$b.log; rc=$?
  echo "[batch $b] rc=$rc $(python3 -c "import json,sys;d=json.load(open('gpurun_out/bs_$b.json'));print('%.3g rec/s step %.3fms split %s fire %.2fms'%(d['value'],d['ms_per_step'],{k:round(x,2) for k,x in d['ingest_split_ms'].items()},d['fire']['ms']))" 2>&1)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/bs_$b.log; exit $rc; fi
done
exit 0
