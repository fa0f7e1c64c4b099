#!/bin/bash
# parity tests (v2 default path), then bench v2 vs v1 in separate processes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/bench_v2.json 2> gpurun_out/bench_v2.log; rc=$?
echo "bench v2 rc=$rc"; tail -n 3 gpurun_out/bench_v2.log; cat gpurun_out/bench_v2.json
if [ $rc -ne 0 ]; then exit $rc; fi
FWA_INGEST=v1 timeout -k 10 300 python -u bench.py --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/bench_v1.json 2> gpurun_out/bench_v1.log; rc=$?
echo "bench v1 rc=$rc"; cat gpurun_out/bench_v1.json
