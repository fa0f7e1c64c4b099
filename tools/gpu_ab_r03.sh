#!/bin/bash
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
echo "== r03 tree"; (cd _ab_r03 && timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu "tests/test_gpu_parity.py::test_random_streams_vs_oracle" -x 2>&1 | tail -4)
echo "== r04 tree"; timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu "tests/test_gpu_parity.py::test_random_streams_vs_oracle" tests/test_narrow_gpu.py tests/test_bench_shapes_gpu.py 2>&1 | tail -12
for o in 0 1 2 3; do
echo "== bench exp=$o"; timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie --no-wire --option 99=$o 2>gpurun_out/ab_bench_$o.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['ingest_split_ms'], d['fire'], d['roofline']['replay_records'])" || exit 1
done
BENCH_ARGS="--option 99=3" bash tools/gpu_pprof.sh
