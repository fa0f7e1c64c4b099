"""Print the tail of a rocprofv3 kernel trace as a timeline (start, gap to previous end, duration)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
sel = rows[-int(sys.argv[2]) if len(sys.argv) > 2 else -40:]
t0 = int(sel[0]["Start_Timestamp"])
prev = None
busy = 0
for r in sel:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev else 0
    busy += e - s
    print("%9.1f gap %7.1f dur %7.1f %s" % ((s - t0) / 1000, gap, (e - s) / 1000, r["Kernel_Name"][:40]))
    prev = e
print("busy %.1f us of %.1f us" % (busy / 1000, (prev - t0) / 1000))
