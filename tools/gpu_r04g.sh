#!/bin/bash
# r04: sliding-fire rewrite (unconditional loads, prefetch, non-temporal rows) A/B + string keys + DECIMAL GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_keydict_strings_gpu.py tests/test_decimal_gpu.py > gpurun_out/r04g_tests1.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r04g_tests1.log | tail -20
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py tests/test_bench_shapes_gpu.py -k "c3 or slide or conservation or hop" > gpurun_out/r04g_tests2.log 2>&1; rc2=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r04g_tests2.log | tail -10
[ $rc2 -gt 1 ] && exit $rc2
for v in 0 1 2 3; do
  echo "== bench c3 slide variant $v"
  timeout -k 10 300 python -u bench.py --config c3 --steps 12 --warmup 2 --no-cpu-baseline --no-pcie --no-wire --option 98=$v \
    2>gpurun_out/r04g_bench.log | tee gpurun_out/r04g_c3_v$v.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4g'%d['value'], '%.3f'%d['ms_per_step'], {k: round(v,3) for k,v in d['ingest_split_ms'].items()}, 'fire/step', round(d['fire']['ms']/12,3))" || { tail -5 gpurun_out/r04g_bench.log; exit 1; }
done
exit $((rc + rc2))
