#!/bin/bash
# r04: session cell pre-aggregation (sessions4.inc): session GPU tests, C5s bench + per-dispatch trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_sessions_gpu.py > gpurun_out/r04h_tests.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed|Error" gpurun_out/r04h_tests.log | tail -20
[ $rc -gt 1 ] && exit $rc
[ $rc -ne 0 ] && exit $rc
echo "== bench c5s"
timeout -k 10 300 python -u bench.py --config c5s --steps 12 --warmup 2 --no-cpu-baseline --no-pcie --no-wire \
  2>gpurun_out/r04h_bench.log | tee gpurun_out/r04h_c5s.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4g'%d['value'], '%.3f'%d['ms_per_step'], 'fire/step', round(d['fire']['ms']/12,3), 'rows', d['rows_emitted'])" || { tail -5 gpurun_out/r04h_bench.log; exit 1; }
CFG=c5s TAG=r04_c5s_pa bash tools/gpu_trace.sh || exit 1
