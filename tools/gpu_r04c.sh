#!/bin/bash
# r04: the narrow Phase P / A kernels and the asynchronous watermark step: parity tests, then C2 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
echo "== r04 tests"; timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_narrow_gpu.py tests/test_bench_shapes_gpu.py tests/test_async_watermark_gpu.py > gpurun_out/r04c_pytest.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r04c_pytest.log | tail -15
[ $rc -gt 1 ] && exit $rc
for o in "--option 99=0 --sync-fire" "--option 99=3 --sync-fire" "--option 99=1 --sync-fire" "--option 99=2 --sync-fire" "--option 99=3"; do
echo "== bench $o"; timeout -k 10 300 python -u bench.py --steps 12 --warmup 2 --no-cpu-baseline --no-pcie --no-wire $o 2>gpurun_out/r04c_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4g'%d['value'], '%.3f'%d['ms_per_step'], {k: round(v,3) for k,v in d['ingest_split_ms'].items()}, round(d['fire']['ms'],2), d['roofline']['replay_records'])" || { tail -5 gpurun_out/r04c_bench.log; exit 1; }
done
BENCH_ARGS="--option 99=3" bash tools/gpu_pprof.sh
