#!/bin/bash
# SQ counters of the C5s cell pre-aggregation kernels (one pass, 8 SQ counters).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU -d $R/gpurun_out/sq_s4 -o run --output-format csv -- python3 $R/bench.py --config c5s --steps 2 --warmup 1 --no-cpu-baseline --no-pcie --no-wire > $R/gpurun_out/sq_s4.log 2>&1; rc=$?; echo rc=$rc
[ $rc -ne 0 ] && { tail -5 $R/gpurun_out/sq_s4.log; exit $rc; }
python3 - <<'P'
import csv, glob, collections, re
f = glob.glob('/root/repo/gpurun_out/sq_s4/**/*counter_collection.csv', recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    m = re.search(r's4_\w+(<[^>]*>)?', r["Kernel_Name"])
    if m: agg[m.group(0)][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():   # fractions of wave cycles; bank conflicts per active-instruction cycle
    wc = d["SQ_WAVE_CYCLES"]
    print("%-26s waves %.3g wait_any %.2f wait_inst %.2f (lds-issue %.2f) active %.2f bankconf/active %.2f" % (
        k, d["SQ_WAVES"], d["SQ_WAIT_ANY"] / wc, d["SQ_WAIT_INST_ANY"] / wc, d["SQ_WAIT_INST_LDS"] / wc,
        d["SQ_ACTIVE_INST_ANY"] / wc, d["SQ_LDS_BANK_CONFLICT"] / max(1.0, d["SQ_ACTIVE_INST_ANY"])))
P
