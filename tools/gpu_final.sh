#!/bin/bash
# Round-end evidence: parity tests + smoke + default bench (driver command), rocprofv3 kernel stats of
# the same bench, then the other BASELINE configs. Stops at the first failing GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-final}
bash tools/gpu_round.sh > gpurun_out/round_$TAG.log 2>&1 || { tail -30 gpurun_out/round_$TAG.log; exit 1; }
grep -E "passed|failed|smoke ok|rc=" gpurun_out/round_$TAG.log
grep '^{' gpurun_out/bench.log > gpurun_out/bench_$TAG.json; cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $R/gpurun_out/rocprof_$TAG -o run --output-format csv -- python3 $R/bench.py --steps 14 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1 || exit 1
f=$(find $R/gpurun_out/rocprof_$TAG -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -8
cd $R
CONFIGS="c3 c4 c5 c5s" bash tools/gpu_configs.sh > gpurun_out/configs_$TAG.log 2>&1 || { tail -20 gpurun_out/configs_$TAG.log; exit 1; }
grep -o '"metric": "[^"]*"\|"value": [0-9.e+]*' gpurun_out/configs_$TAG.log
exit 0
