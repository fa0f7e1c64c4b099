#!/bin/bash
# SQ counters of the C5s cell pre-aggregation kernels (one pass, 8 SQ counters).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_VALU -d $R/gpurun_out/sq_s4 -o run --output-format csv -- python3 $R/bench.py --config c5s --steps 2 --warmup 1 --no-cpu-baseline --no-pcie --no-wire > $R/gpurun_out/sq_s4.log 2>&1; rc=$?; echo rc=$rc
[ $rc -ne 0 ] && { tail -5 $R/gpurun_out/sq_s4.log; exit $rc; }
python3 - <<'P'
import csv, glob, collections
f = glob.glob('/root/repo/gpurun_out/sq_s4/**/*counter_collection.csv', recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    if "s4_" not in n: continue
    k = n.split("(")[0].split("::")[-1][:40]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k, {c: "%.3g" % v for c, v in sorted(d.items())})
P
