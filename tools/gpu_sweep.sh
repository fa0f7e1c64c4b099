#!/bin/bash
# parity tests + bench under several env settings (one process each)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -n "$PYTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -n 8 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
i=0
IFS=';' read -ra VARIANTS <<< "${VARIANTS:-base}"
for v in "${VARIANTS[@]}"; do
  i=$((i+1))
  env $( [ "$v" != "base" ] && echo $v ) timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---steps 6 --warmup 1 --no-cpu-baseline} > gpurun_out/sweep_$i.json 2> gpurun_out/sweep_$i.log; rc=$?
  echo "[$v] rc=$rc $(python3 -c "import json,sys;d=json.load(open('gpurun_out/sweep_$i.json'));print('%.3g rec/s step %.3fms split %s fire %.2fms'%(d['value'],d['ms_per_step'],{k:round(x,2) for k,x in d['ingest_split_ms'].items()},d['fire']['ms']))" 2>&1)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/sweep_$i.log; exit $rc; fi
done
exit 0
