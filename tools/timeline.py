"""Merge a rocprofv3 kernel trace and HIP API trace into one timeline around the last two launches of
a kernel (default partition): python tools/timeline.py <rocprof dir> [kernel substring]."""
import csv
import os
import re
import sys

d = sys.argv[1]
needle = sys.argv[2] if len(sys.argv) > 2 else "partition"
k = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
hp = os.path.join(d, "run_hip_api_trace.csv")
h = list(csv.DictReader(open(hp))) if os.path.exists(hp) else []
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
       "GPU " + re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])[:34]) for r in k]
skip = set("hipGetLastError hipSetDevice hipGetDevice hipPeekAtLastError hipDeviceGetAttribute hipGetDeviceCount "
           "hipCtxGetCurrent hipStreamGetCaptureInfo hipStreamIsCapturing hipPointerGetAttributes "
           "hipDevicePrimaryCtxGetState hipGetDeviceProperties hipGetDevicePropertiesR0600 hipEventElapsedTime".split())
ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "   host " + r["Function"]) for r in h
       if r["Function"] not in skip]
ev.sort()
idx = [i for i, e in enumerate(ev) if needle in e[2] and e[2].startswith("GPU")]
a, b = idx[-2], idx[-1]
t0 = ev[a][0]
gpu_busy = 0
for e in ev[a:b]:
    print("%9.1f %8.1f %s" % ((e[0] - t0) / 1000, (e[1] - e[0]) / 1000, e[2]))
    if e[2].startswith("GPU"):
        gpu_busy += e[1] - e[0]
print("step %.1f us, GPU busy %.1f us" % ((ev[b][0] - t0) / 1000, gpu_busy / 1000))
