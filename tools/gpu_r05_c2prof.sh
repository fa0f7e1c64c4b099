#!/bin/bash
# r05: C2 kernel traces, synchronous and asynchronous watermark step (GPU idle gaps), then SQ counters of the ingest kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r05_c2_sync BENCH_ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-pcie --no-wire" bash tools/gpu_trace.sh || exit 1
TAG=r05_c2_async BENCH_ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-pcie --no-wire --async-fire" bash tools/gpu_trace.sh || exit 1
for t in sync async; do echo "== $t"; python3 tools/trace_gaps.py gpurun_out/tr_r05_c2_${t}_kernel_trace.csv 40 | tail -42; done
TAG=r05_sq_c2 bash tools/gpu_sq.sh
