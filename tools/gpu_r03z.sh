#!/bin/bash
# Round-3 closing evidence: whole GPU suite + smoke + C2 trace (gpu_full.sh), then the other configs' bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r03z bash tools/gpu_full.sh && bash tools/gpu_r03_configs.sh
