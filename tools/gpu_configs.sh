#!/bin/bash
# Short bench runs of the non-headline BASELINE configs (C3/C4/C5/C5-session) at N=1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for c in ${CONFIGS:-c4 c5 c5s}; do
  timeout -k 10 ${TO:-300} python -u bench.py --config $c ${BENCH_ARGS:---steps 6 --warmup 1} > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.log
  rc=$?
  echo "== $c rc=$rc"; cat gpurun_out/bench_$c.json; tail -n 5 gpurun_out/bench_$c.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
