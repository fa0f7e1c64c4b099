#!/bin/bash
# r04: decimal + skew re-check, then the narrow kernels / async watermark A/B on C2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_decimal_gpu.py tests/test_skew_gpu.py tests/test_narrow_gpu.py tests/test_bench_shapes_gpu.py \
  tests/test_async_watermark_gpu.py tests/test_operators_gpu.py > gpurun_out/r04e_tests.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r04e_tests.log | tail -30
[ $rc -gt 1 ] && exit $rc
for o in "--option 99=0 --sync-fire" "--option 99=3 --sync-fire" "--option 99=1 --sync-fire" "--option 99=2 --sync-fire" "--option 99=0" "--option 99=3"; do
echo "== bench $o"; timeout -k 10 300 python -u bench.py --steps 12 --warmup 2 --no-cpu-baseline --no-pcie --no-wire $o 2>gpurun_out/r04e_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4g'%d['value'], '%.3f'%d['ms_per_step'], {k: round(v,3) for k,v in d['ingest_split_ms'].items()}, round(d['fire']['ms'],2), d['roofline']['replay_records'])" || { tail -5 gpurun_out/r04e_bench.log; exit 1; }
done
BENCH_ARGS="--option 99=3" bash tools/gpu_pprof.sh
