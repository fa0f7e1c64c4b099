#!/bin/bash
# Flat Phase P layout: parity suites, then C2 / C3 / C5 bench A/B (FWA_FLAT=0: sub-buckets) and a Phase P clock profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest --maxfail 10 -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_skew_gpu.py tests/test_bench_shapes_gpu.py tests/test_snapshot_gpu.py tests/test_distributed_gpu.py \
  tests/test_late_firing_gpu.py tests/test_sql_nulls_gpu.py > gpurun_out/flat_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/flat_pytest.log | tail -15
[ $rc -ne 0 ] && exit $rc
for cfg in c2 c3 c5; do for f in 1 0; do
  w=1; [ $cfg = c3 ] && w=2
  FWA_FLAT=$f timeout -k 10 300 python3 bench.py --config $cfg --steps 12 --warmup $w --no-cpu-baseline --no-pcie --no-wire > gpurun_out/flat_${cfg}_$f.json 2> gpurun_out/flat_${cfg}_$f.log || { tail -5 gpurun_out/flat_${cfg}_$f.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/flat_${cfg}_$f.json')); s=d['ingest_split_ms']; L=d['roofline']['launches']; print('$cfg flat=$f', round(d['value']/1e9,2), round(d['ms_per_step'],3), 'P', round(s['partition']/L,3), 'A', round(s['combine']/L,3), 'frac', round(d['roofline']['frac'],4))"
done; done
FWA_PPROF=1 timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-pcie --no-wire > gpurun_out/flat_pprof.json 2> gpurun_out/flat_pprof.log || exit 1
grep pprof gpurun_out/flat_pprof.log | tail -2
