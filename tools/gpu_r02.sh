#!/bin/bash
# Round-2 GPU sequence: parity tests -> smoke -> default bench (the driver's command) -> rocprofv3 kernel
# stats of the same bench. Every GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-r02}
STEPS=${STEPS:-pytest,smoke,bench,prof}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1; local rc=$?
  echo "== $name rc=$rc $(date +%T)"; tail -n 30 "gpurun_out/${name}_$TAG.log"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
}
[[ $STEPS == *pytest* ]] && run pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
[[ $STEPS == *smoke* ]] && run smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* ]] && run bench 600 python -u bench.py ${BENCH_ARGS}
[[ $STEPS == *bench* ]] && { grep '^{' gpurun_out/bench_$TAG.log > gpurun_out/bench_$TAG.json || true; }
if [[ $STEPS == *prof* ]]; then
  cd /tmp && export TMPDIR=/tmp
  run_prof() { timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/rocprof_$TAG -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-pcie ${BENCH_ARGS}; }
  echo "== prof $(date +%T)"
  run_prof > $R/gpurun_out/prof_$TAG.log 2>&1; rc=$?
  echo "== prof rc=$rc"; tail -5 $R/gpurun_out/prof_$TAG.log
  [ $rc -ne 0 ] && exit $rc
  f=$(find $R/gpurun_out/rocprof_$TAG -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-4 "$f" | head -12
fi
exit 0
