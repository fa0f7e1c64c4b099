#!/bin/bash
# r04: string/DECIMAL/slide tests, sliding-fire clear-mode A/B, session pre-aggregation tests + C5s
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_keydict_strings_gpu.py tests/test_decimal_gpu.py tests/test_gpu_parity.py tests/test_bench_shapes_gpu.py \
  -k "not (test_gpu_parity and not (c3 or slide or conservation or hop)) and not (bench_shapes and not c3)" > gpurun_out/r04j_tests1.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r04j_tests1.log | tail -12
[ $rc -gt 1 ] && exit $rc
for v in 0 1 2; do
  echo "== bench c3 clear variant $v"
  timeout -k 10 300 python -u bench.py --config c3 --steps 12 --warmup 2 --no-cpu-baseline --no-pcie --no-wire --option 98=$v \
    2>gpurun_out/r04j_bench.log | tee gpurun_out/r04j_c3_v$v.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4g'%d['value'], '%.3f'%d['ms_per_step'], {k: round(v,3) for k,v in d['ingest_split_ms'].items()}, 'fire/step', round(d['fire']['ms']/12,3))" || { tail -5 gpurun_out/r04j_bench.log; exit 1; }
done
bash tools/gpu_r04h.sh
