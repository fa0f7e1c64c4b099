#!/bin/bash
# r04: HBM-traffic PMC passes over every config (tools/gpu_pmc_all.sh) and their summaries (profiles/r04_pmc_<cfg>.json)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CFGS="${CFGS:-c2 c3 c4 c5 c5s}" bash tools/gpu_pmc_all.sh || exit $?
python3 tools/pmc_summary.py gpurun_out/pmca r04 3 2>&1 | tail -30
mkdir -p gpurun_out/pmc_json && cp profiles/r04_pmc_*.json gpurun_out/pmc_json/ 2>/dev/null; ls gpurun_out/pmc_json
