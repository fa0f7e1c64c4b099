#!/bin/bash
# Phase P / Phase A per-phase clock profiles (fwa_set_option FWA_OPT_PROFILE) on C2 (BENCH_ARGS: extra bench flags).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-pcie --no-wire --option profile=1 $BENCH_ARGS \
  > gpurun_out/prof_phases.json 2> gpurun_out/prof_phases.log || { tail -5 gpurun_out/prof_phases.log; exit 1; }
grep -E "pprof|aprof" gpurun_out/prof_phases.log | tail -8
