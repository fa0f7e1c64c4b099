#!/bin/bash
# Phase P timing ablation: reservation atomics replaced by a constant (wrong results) vs the real kernel, clock profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for ab in 0 1; do
  FWA_PABL=$ab FWA_PPROF=1 timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-pcie --no-wire --no-cpu-baseline > gpurun_out/pabl$ab.json 2> gpurun_out/pabl$ab.log || { tail -20 gpurun_out/pabl$ab.log; exit 1; }
  echo "abl $ab"; grep "\[pprof\]" gpurun_out/pabl$ab.log | tail -2
done
