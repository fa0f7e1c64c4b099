#!/bin/bash
# The whole GPU parity suite with every eligible TUMBLE handle forced onto record lists (--force-record-lists), minus the
# tests that assert dense-layout internals (replay counts, the layout choice itself).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --force-record-lists --timeout 200 --timeout-method thread -p no:cacheprovider \
  -k "not dense and not auto_selected and not switches_to_pre_aggregation" > gpurun_out/record_lists_suite.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/record_lists_suite.log | tail -20
exit $rc
