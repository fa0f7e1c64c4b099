#!/bin/bash
# HBM-traffic PMC passes (FETCH_SIZE; WRITE_SIZE, one counter per run) over the C2 bench's wire-input leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/pmcw
cd /tmp && export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $ctr -T -d $R/gpurun_out/pmcw/$ctr -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pcie --wire-batches 3 > $R/gpurun_out/pmcw/$ctr.log 2>&1; rc=$?
  echo "$ctr rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $R/gpurun_out/pmcw/$ctr.log; exit $rc; fi
done
exit 0
