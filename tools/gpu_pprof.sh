#!/bin/bash
# Phase P / Phase A per-phase clock profiles (FWA_PPROF / FWA_APROF) on C2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
FWA_PPROF=1 timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-pcie --no-wire > gpurun_out/pprof.json 2> gpurun_out/pprof.log || { tail -5 gpurun_out/pprof.log; exit 1; }
grep pprof gpurun_out/pprof.log | tail -4
FWA_APROF=1 timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-pcie --no-wire > gpurun_out/aprof.json 2> gpurun_out/aprof.log || { tail -5 gpurun_out/aprof.log; exit 1; }
grep aprof gpurun_out/aprof.log | tail -4
