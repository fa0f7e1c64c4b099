#!/bin/bash
# SQ counters of the N>1 plan's drain-route and owner kernels (tools/partials_cost.py) (one rocprofv3 --pmc pass per counter group, each under its own kill
# timeout), summarised per kernel family matching KRE; TAG names the output.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
TAG=${TAG:-sq_owner}; KRE=${KRE:-"(mf_part|mf_merge|drain_route)_kernel"}
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU" \
            "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES"; do
  i=$((i+1))
  rm -rf $R/gpurun_out/${TAG}_p$i
  timeout -s KILL 120 rocprofv3 --pmc $pass -d $R/gpurun_out/${TAG}_p$i -o run --output-format csv -- python3 $R/tools/partials_cost.py --order merge_fire --steps 4 \
    > $R/gpurun_out/${TAG}_p$i.log 2>&1; rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/${TAG}_p$i.log; exit $rc; }
done
cd $R
python3 - "$TAG" "$KRE" <<'P'
import csv, glob, collections, re, sys
tag, kre = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob('gpurun_out/%s_p*/**/*counter_collection.csv' % tag, recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(kre, r["Kernel_Name"])
        if m: agg[m.group(0)][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in sorted(agg.items()):
    wc = d["SQ_WAVE_CYCLES"] or 1
    print("%-22s waves %.3g | wave-cycle fractions: wait_any %.2f wait_inst %.2f (lds %.2f) active %.2f | "
          "lds-bank-conflict/active-lds %.2f | per wave: valu %.0f lds %.0f vmem_rd %.0f vmem_wr %.0f salu %.0f" % (
        k, d["SQ_WAVES"] / 2, d["SQ_WAIT_ANY"] / wc, d["SQ_WAIT_INST_ANY"] / wc, d["SQ_WAIT_INST_LDS"] / wc,
        d["SQ_ACTIVE_INST_ANY"] / wc, d["SQ_LDS_BANK_CONFLICT"] / max(1.0, d["SQ_ACTIVE_INST_LDS"]),
        d["SQ_INSTS_VALU"] / max(1, d["SQ_WAVES"] / 2), d["SQ_INSTS_LDS"] / max(1, d["SQ_WAVES"] / 2),
        d["SQ_INSTS_VMEM_RD"] / max(1, d["SQ_WAVES"] / 2), d["SQ_INSTS_VMEM_WR"] / max(1, d["SQ_WAVES"] / 2),
        d["SQ_INSTS_SALU"] / max(1, d["SQ_WAVES"] / 2)))
P
