#!/bin/bash
# Kernel trace of tools/partials_cost.py (the N>1 two-phase plan's per-step pieces on one GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-pc}
timeout -k 10 300 python3 tools/partials_cost.py $PC_ARGS > gpurun_out/${TAG}_plain.log 2>&1 || { tail -20 gpurun_out/${TAG}_plain.log; exit 1; }
cat gpurun_out/${TAG}_plain.log
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/tr_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tr_$TAG -o run --output-format csv -- \
  python3 $R/tools/partials_cost.py $PC_ARGS > $R/gpurun_out/tr_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/tr_$TAG.log; exit 1; }
cd $R
s=$(find gpurun_out/tr_$TAG -name "*kernel_stats.csv" | head -1)
f=$(find gpurun_out/tr_$TAG -name "*kernel_trace.csv" | head -1)
cp "$s" gpurun_out/tr_${TAG}_kernel_stats.csv
cp "$f" gpurun_out/tr_${TAG}_kernel_trace.csv
cut -d, -f1-8 gpurun_out/tr_${TAG}_kernel_stats.csv | head -40
