#!/bin/bash
# PMC passes (one counter group per run, each under its own kill timeout) over a short bench run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
ARGS=${PMC_ARGS:---steps 2 --warmup 1 --no-cpu-baseline}
i=0
IFS=';' read -ra PASSES <<< "${PASSES:-FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS;TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE}"
for pass in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass -T -d $R/gpurun_out/pmc/p$i -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc/p$i.log 2>&1; rc=$?
  echo "pass $i [$pass] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $R/gpurun_out/pmc/p$i.log; exit $rc; fi
done
exit 0
