#!/bin/bash
# Instruction-mix PMC passes (combine / partition kernels) for two bench configs, one counter group per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/pmcc
cd /tmp && export TMPDIR=/tmp
for cfg in ${CFGS:-c2 c3}; do
  i=0
  IFS=';' read -ra PASSES <<< "${PASSES:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES;SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_LDS}"
  for pass in "${PASSES[@]}"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $pass -T -d $R/gpurun_out/pmcc/${cfg}_p$i -o run --output-format csv -- python3 $R/bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-pcie > $R/gpurun_out/pmcc/${cfg}_p$i.log 2>&1; rc=$?
    echo "$cfg pass $i [$pass] rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $R/gpurun_out/pmcc/${cfg}_p$i.log; exit $rc; fi
  done
done
exit 0
