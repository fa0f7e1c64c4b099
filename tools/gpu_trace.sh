#!/bin/bash
# Per-dispatch rocprofv3 kernel trace of the driver's bench command and the roofline recomputed from it
# (tools/roofline_from_trace.py). TAG names the output; CFG the bench config (default c2);
# BENCH_ARGS the bench flags (default: the driver's `--gpus 1 --steps 20 --warmup 5`).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-trace}
CFG=${CFG:-c2}
ARGS=${BENCH_ARGS:---gpus 1 --steps 20 --warmup 5}
[ "$CFG" != c2 ] && ARGS="$ARGS --config $CFG"
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/tr_$TAG
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tr_$TAG -o run --output-format csv -- \
  python3 $R/bench.py $ARGS > $R/gpurun_out/tr_$TAG.json 2> $R/gpurun_out/tr_$TAG.log || { tail -20 $R/gpurun_out/tr_$TAG.log; exit 1; }
cd $R
cat gpurun_out/tr_$TAG.json
f=$(find gpurun_out/tr_$TAG -name "*kernel_trace.csv" | head -1)
s=$(find gpurun_out/tr_$TAG -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/tr_${TAG}_kernel_trace.csv
cp "$s" gpurun_out/tr_${TAG}_kernel_stats.csv
python3 tools/roofline_from_trace.py "$f" gpurun_out/tr_$TAG.json --out gpurun_out/tr_${TAG}_roofline.json | \
  python3 -c "import json,sys; d=json.load(sys.stdin); print(json.dumps({k: d[k] for k in ('dominant','step') if k in d}, indent=1)); print(json.dumps(d.get('fire')))"
