#!/bin/bash
# Reduce-path GPU check: the reduction / parity / ABI tests, then the reduce bench line (gpurun_out/<TAG>_*).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r06_reduce}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_reduce_gpu.py \
  tests/test_abi.py tests/test_gpu_parity.py > gpurun_out/${T}_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config reduce ${BENCH_ARGS} > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || { tail -5 gpurun_out/${T}_bench.log; exit 1; }
python3 - "$T" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/%s_bench.json" % sys.argv[1]).read().strip().splitlines()[-1])
print("reduce %.2f G rec/s %.3f ms/step ingest %.3f ms/launch fire %.3f ms/step frac %.4f" % (
    d["value"] / 1e9, d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline_fire"]["ms_per_step"],
    d["roofline"]["frac"]))
PY
