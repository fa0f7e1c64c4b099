#!/bin/bash
# Short C2 bench under several env settings (one process each): phase split per setting.
# VARIANTS: ';'-separated env assignments, e.g. "FWA_AABL=1;FWA_PABL=2"; "" = baseline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
IFS=';' read -ra VS <<< "${VARIANTS:-}"
VS=("BASE=1" "${VS[@]}")
i=0
for v in "${VS[@]}"; do
  i=$((i+1))
  env $v timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---steps 6 --warmup 1 --no-cpu-baseline} > gpurun_out/ev_$i.json 2> gpurun_out/ev_$i.log; rc=$?
  echo "[$v] rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/ev_$i.json'));print('%.4g rec/s step %.3fms part %.3f comb %.3f fire %.3f'%(d['value'],d['ms_per_step'],d['ingest_split_ms']['partition']/d['roofline']['launches'],d['ingest_split_ms']['combine']/d['roofline']['launches'],d['fire']['ms']/max(1,d['fire']['launches'])))" 2>&1)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ev_$i.log; exit $rc; fi
done
exit 0
