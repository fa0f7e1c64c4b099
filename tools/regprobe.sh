#!/bin/bash
# VGPR / spill table of the ingest kernels (tools/regprobe.hip). Extra hipcc flags pass through, e.g. -DFWA_MP_IT=4.
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -c tools/regprobe.hip -o /tmp/regprobe.o \
  -Rpass-analysis=kernel-resource-usage "$@" 2>&1 | python3 -c '
import re, subprocess, sys
cur = None; rows = []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()}
        cur["name"] = re.sub(r"\(anonymous namespace\)::|\(.*", "", cur["name"]).replace("void ", ""); rows.append(cur); continue
    m = re.search(r"remark:\s+(VGPRs Spill|SGPRs Spill|VGPRs|ScratchSize)[^:]*: (\d+)", line)
    if m and cur is not None: cur[m.group(1)] = int(m.group(2))
bad = 0
for r in sorted(rows, key=lambda r: r["name"]):
    print("%s %-48s VGPR %3d  VGPR-spill %3d  SGPR-spill %3d  scratch %3d" % ("*" if r.get("VGPRs Spill", 0) else " ", r["name"], r.get("VGPRs", -1), r.get("VGPRs Spill", -1), r.get("SGPRs Spill", -1), r.get("ScratchSize", -1)))
    bad += r.get("VGPRs Spill", 0) > 0
print("%d of %d kernels spill VGPRs" % (bad, len(rows)))
'
