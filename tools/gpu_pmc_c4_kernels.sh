#!/bin/bash
# Per-kernel HBM traffic of the C4 record-list kernels: FETCH_SIZE and WRITE_SIZE passes (one counter per run, each
# under its own kill timeout); per-kernel averages printed by tools/pmc_kernels.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/pmck
cd /tmp && export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $ctr -T -d $R/gpurun_out/pmck/c4_$ctr -o run --output-format csv -- python3 $R/bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --no-wire > $R/gpurun_out/pmck/c4_$ctr.log 2>&1; rc=$?
  echo "c4 $ctr rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $R/gpurun_out/pmck/c4_$ctr.log; exit $rc; fi
done
python3 $R/tools/pmc_kernels.py $R/gpurun_out/pmck
