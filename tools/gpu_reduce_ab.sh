#!/bin/bash
# Reduce-path A/B on one box: the reduce tests, then the reduce bench alternating ingest variants (VARIANTS, default
# "0 16": bit 16 loads the record-index column in partition3 instead of computing it), then C5 (shares partition3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r06_reduce_ab}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_reduce_gpu.py \
  > gpurun_out/${T}_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in ${VARIANTS:-0 16}; do
    timeout -k 10 300 python bench.py --config reduce --no-cpu-baseline --option ingest_variant=$v > gpurun_out/${T}_v${v}_$r.json \
      2> gpurun_out/${T}_v${v}_$r.log || { tail -5 gpurun_out/${T}_v${v}_$r.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/${T}_v${v}_$r.json').read().strip().splitlines()[-1]); print('reduce v$v run $r', round(d['value']/1e9,3), 'G rec/s', round(d['ms_per_step'],3), 'ms/step ingest', round(d['roofline']['avg_launch_ms'],3))"
  done
done
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-pcie --no-wire --no-wide > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.log || { tail -5 gpurun_out/${T}_c5.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/${T}_c5.json').read().strip().splitlines()[-1]); print('c5', round(d['value']/1e9,3), 'G rec/s', round(d['ms_per_step'],3))"
