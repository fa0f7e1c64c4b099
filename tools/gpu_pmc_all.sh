#!/bin/bash
# HBM-traffic PMC passes (FETCH_SIZE; WRITE_SIZE -- one counter per run, each under its own kill timeout) over a
# short bench of every config; summarised by tools/pmc_summary.py into profiles/<tag>_pmc_<cfg>.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/pmca
cd /tmp && export TMPDIR=/tmp
for cfg in ${CFGS:-c2 c3 c4 c5 c5s}; do
  W=1; [ $cfg = c3 ] && W=2
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $ctr -T -d $R/gpurun_out/pmca/${cfg}_$ctr -o run --output-format csv -- python3 $R/bench.py --config $cfg --steps 3 --warmup $W --no-cpu-baseline --no-pcie --no-wire --no-wide > $R/gpurun_out/pmca/${cfg}_$ctr.log 2>&1; rc=$?
    echo "$cfg $ctr rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $R/gpurun_out/pmca/${cfg}_$ctr.log; exit $rc; fi
  done
done
exit 0
