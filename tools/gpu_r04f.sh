#!/bin/bash
# r04: C3 (sliding fire clears retiring slices) and C5s: per-dispatch traces + roofline, C3 HBM-traffic PMC passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py tests/test_bench_shapes_gpu.py tests/test_record_lists_gpu.py tests/test_keydict_gpu.py \
  -k "c3 or slide or conservation or record or c4 or keydict or dict" > gpurun_out/r04f_tests.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r04f_tests.log | tail -10
[ $rc -gt 1 ] && exit $rc
for c in c2 c3 c4; do
  echo "== bench $c"; timeout -k 10 300 python -u bench.py --config $c --steps 12 --warmup 2 --no-cpu-baseline --no-pcie --no-wire 2>gpurun_out/r04f_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4g'%d['value'], '%.3f'%d['ms_per_step'], {k: round(v,3) for k,v in d['ingest_split_ms'].items()}, round(d['fire']['ms'],2))" || { tail -5 gpurun_out/r04f_bench.log; exit 1; }
done
CFG=c3 TAG=r04_c3 bash tools/gpu_trace.sh || exit 1
CFG=c5s TAG=r04_c5s bash tools/gpu_trace.sh || exit 1
CFGS=c3 bash tools/gpu_pmc_all.sh || exit 1
python3 tools/pmc_summary.py gpurun_out/pmca r04 3 2>&1 | tail -20
