#!/bin/bash
# r04: gpu_r04g (strings, DECIMAL, sliding-fire A/B) then gpu_r04h (session pre-aggregation)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r04g.sh || exit $?
bash tools/gpu_r04h.sh
