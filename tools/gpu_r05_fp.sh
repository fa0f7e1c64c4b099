#!/bin/bash
# r05: combiner fingerprint probes (FWA_OPT_INGEST_VARIANT bit 1): parity with the variant forced, then C2 A/B x2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_bench_shapes_gpu.py --force-option ingest_variant=2 > gpurun_out/r05_fp_parity.log 2>&1 || { tail -30 gpurun_out/r05_fp_parity.log; exit 1; }
tail -2 gpurun_out/r05_fp_parity.log
for rep in 1 2; do for v in 0 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie --no-wire --option ingest_variant=$v > gpurun_out/r05_fp_v${v}_$rep.json 2> gpurun_out/r05_fp_v${v}_$rep.log || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r05_fp_v${v}_$rep.json').read().strip().splitlines()[-1]); r=d['roofline']; print('v$v rep$rep', round(d['value']/1e9,2), round(d['ms_per_step'],4), round(r['frac'],4))"
done; done
