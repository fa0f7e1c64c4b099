#!/bin/bash
# r04: per-record Phase P / Phase A cost vs batch size (do MALL-resident buckets help?)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BATCHES="2097152 4194304 8388608 16777216 67108864" RECS=536870912 bash tools/gpu_batchsweep.sh
