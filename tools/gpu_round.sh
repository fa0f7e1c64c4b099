#!/bin/bash
# GPU-box sequence: parity tests -> smoke -> short bench. Stops at the first crash/timeout
# (exit codes other than 0/1), never retries a GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
STEPS=${STEPS:-pytest,smoke,bench}
[[ $STEPS == *pytest* ]] && step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
[[ $STEPS == *smoke* ]] && step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* ]] && step bench 600 python -u bench.py ${BENCH_ARGS:---steps 4 --warmup 1 --no-cpu-baseline}
exit 0
