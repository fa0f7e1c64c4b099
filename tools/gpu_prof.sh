#!/bin/bash
# quick parity + bench + rocprofv3 kernel-trace stats of a short bench run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-prof}
if [ -n "$PYTEST" ] || [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread $PYTEST ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -n 15 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---steps 6 --warmup 1 --no-cpu-baseline} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json
if [ $rc -ne 0 ]; then tail gpurun_out/bench_$TAG.log; exit $rc; fi
if [ -z "$NOPROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $GRAFT_REPO_ROOT/gpurun_out/rocprof_$TAG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py ${PROF_ARGS:---steps 3 --warmup 1 --no-cpu-baseline} > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1; rc=$?
  echo "rocprof rc=$rc"
  f=$(find $GRAFT_REPO_ROOT/gpurun_out/rocprof_$TAG -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cut -d, -f1-8 "$f" | head -20
fi
exit 0
