#!/bin/bash
# A/B of an ingest variant (FWA_OPT_INGEST_VARIANT=$V) against the default on C2: parity with the variant forced
# (test_gpu_parity + test_bench_shapes), then REPS alternating bench runs. TAG names the outputs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=${V:?variant}; TAG=${TAG:-ab}; REPS=${REPS:-2}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_bench_shapes_gpu.py --force-option ingest_variant=$V > gpurun_out/${TAG}_parity.log 2>&1 || { tail -30 gpurun_out/${TAG}_parity.log; exit 1; }
tail -1 gpurun_out/${TAG}_parity.log
for rep in $(seq $REPS); do for v in 0 $V; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie --no-wire --no-wide --option ingest_variant=$v > gpurun_out/${TAG}_v${v}_$rep.json 2> gpurun_out/${TAG}_v${v}_$rep.log || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_v${v}_$rep.json').read().strip().splitlines()[-1]); s=d['ingest_split_ms']; n=d['steps']; print('v$v rep$rep', round(d['value']/1e9,2), round(d['ms_per_step'],4), 'P %.3f A %.3f' % (s['partition']/n, s['combine']/n))"
done; done
