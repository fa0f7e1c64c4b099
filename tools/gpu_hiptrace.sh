#!/bin/bash
# bench + rocprofv3 kernel trace + HIP API trace (no counters) of a short bench, for host-gap analysis
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-ht}
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---steps 14 --warmup 1 --no-cpu-baseline} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $R/gpurun_out/rocprof_$TAG -o run --output-format csv -- python3 $R/bench.py ${PROF_ARGS:---steps 4 --warmup 1 --no-cpu-baseline} > $R/gpurun_out/prof_$TAG.log 2>&1; rc=$?
echo "rocprof rc=$rc"; ls $R/gpurun_out/rocprof_$TAG
exit $rc
