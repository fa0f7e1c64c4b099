#!/bin/bash
# A/B of Phase P variants (FWA_PDB: next-tile pairs issued during classify), C2 bench lines; parity of the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in 0 1 2 3 0; do
  FWA_PDB=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pcie --no-wire > gpurun_out/ab_pdb$v.json 2> gpurun_out/ab_pdb$v.log || { tail -5 gpurun_out/ab_pdb$v.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_pdb$v.json')); s=d['ingest_split_ms']; n=d['steps']; print('pdb=$v', round(d['value']/1e9,2), round(d['ms_per_step'],3), 'P', round(s['partition']/d['roofline']['launches'],3), 'A', round(s['combine']/d['roofline']['launches'],3), 'frac', round(d['roofline']['frac'],4))"
done
for v in 1 2 3; do
  FWA_PDB=$v timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_bench_shapes_gpu.py tests/test_gpu_parity.py tests/test_skew_gpu.py > gpurun_out/ab_pdb_test$v.log 2>&1 || { tail -20 gpurun_out/ab_pdb_test$v.log; exit 1; }
  tail -1 gpurun_out/ab_pdb_test$v.log
done
