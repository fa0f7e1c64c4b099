#!/bin/bash
# Wire decoder: parity tests, bench C2 line with the wire_input leg, rocprofv3 kernel stats of the same bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
TAG=${TAG:-wire}
timeout -k 10 300 python -u -m pytest tests/test_wire_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wtest_$TAG.log 2>&1 || { tail -30 gpurun_out/wtest_$TAG.log; exit 1; }
tail -2 gpurun_out/wtest_$TAG.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie --steps 4 > gpurun_out/wbench_$TAG.log 2>&1 || { tail -20 gpurun_out/wbench_$TAG.log; exit 1; }
grep '^{' gpurun_out/wbench_$TAG.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['wire_input']))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/wprof_$TAG -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-pcie --steps 4 > $R/gpurun_out/wprof_$TAG.log 2>&1 || { tail -5 $R/gpurun_out/wprof_$TAG.log; exit 1; }
f=$(find $R/gpurun_out/wprof_$TAG -name "*kernel_stats.csv" | head -1); grep -i wire "$f" | cut -d, -f1-4
