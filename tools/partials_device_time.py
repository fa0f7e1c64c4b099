"""Device time per step of tools/partials_cost.py from its rocprofv3 kernel trace: the N=1 engine's kernels against
the N>1 rank's (local pre-aggregator + owner) kernels, by stream, skipping the first `skip` steps (warm-up / region
sizing). Usage: python tools/partials_device_time.py <kernel_trace.csv> [steps] [skip]"""
import csv
import sys

trace = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 2
rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
# streams in order of first use: 0 = torch's (generator / model copies), then the N=1 engine, the local engine, owner(s)
order = []
for r in rows:
    q = r.get("Stream_Id", r.get("Queue_Id"))
    if q not in order:
        order.append(q)
per = {}
for r in rows:
    q = r.get("Stream_Id", r.get("Queue_Id"))
    per.setdefault(q, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
eng = [q for q in order if q != "0"]
single, local, owners = eng[0], eng[1], eng[2:]


# step boundaries: every step starts with the N=1 engine's push (one partition3_kernel each)
marks = [int(r["Start_Timestamp"]) for r in rows
         if r.get("Stream_Id", r.get("Queue_Id")) == single and "partition3_kernel" in r["Kernel_Name"]]
t0 = marks[skip] if len(marks) > skip else 0


def steady(q):
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows
         if r.get("Stream_Id", r.get("Queue_Id")) == q and int(r["Start_Timestamp"]) >= t0]
    return sum(d) / 1e6 / (steps - skip)


n1 = steady(single)
loc = steady(local)
own = [steady(q) for q in owners]
print("device ms per step: N=1 engine %.3f; N>1 rank: local %.3f + owner %s" % (n1, loc, " / ".join("%.3f" % o for o in own)))
for o in own:
    print("  per-rank device time %.3f ms = %.2fx N=1" % (loc + o, (loc + o) / n1))
