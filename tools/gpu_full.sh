#!/bin/bash
# Full default bench (C2 workload, with cpu_baseline) + rocprofv3 kernel stats of the same command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-full}
timeout -k 10 600 python -u bench.py $BENCH_ARGS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.log
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $R/gpurun_out/rocprof_$TAG -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline $BENCH_ARGS > $R/gpurun_out/prof_$TAG.log 2>&1; rc=$?
echo "rocprof rc=$rc"; tail -1 $R/gpurun_out/prof_$TAG.log
f=$(find $R/gpurun_out/rocprof_$TAG -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cut -d, -f1-7 "$f" | head -12
exit 0
