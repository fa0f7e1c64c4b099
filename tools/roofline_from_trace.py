"""Recompute bench.py's `roofline.frac` from a rocprofv3 per-dispatch kernel trace of the same command.

    python tools/roofline_from_trace.py <run_kernel_trace.csv> <bench json line file> [--out profiles/x.json]

The trace is `rocprofv3 --kernel-trace --output-format csv -- python3 bench.py --gpus 1 --steps K --warmup W ...`.
The main engine's calls come first in bench.py (W warm-up steps, then K timed steps; the PCIe and wire legs
create their own engines afterwards), so the timed dispatches of a kernel family are its occurrences
[W, W + K) in dispatch order, counted on the main engine's HIP stream (the stream of the first ingest
dispatch). Only steady-state timed dispatches enter the average: cold dispatches of the warm-up steps and
the side legs are excluded.

Families (regexes over the kernel name):
  ingest (C2/C3/C5): partition3_kernel / partition2_kernel + combine3_kernel (one of each per push),
                    ingest_kernel replays are listed separately;
  push (C4 record lists): sp_range + sp_hist + sp_scan + sp_scatter;  fire: sp_refine + sp_agg;
  sessions (C5s): s5_* / s4_* (cell pre-aggregation) or sess3_* / sess2_* + hipcub radix sort / scan;
  reduce: the ingest family plus iota_kernel and red_iota_payload_kernel.
frac = algorithmic bytes per launch (bench line `roofline.alg_bytes_per_launch`) / average launch time / peak.
"""
import argparse
import csv
import json
import re
import statistics
import sys

FAMILIES = {
    "ingest": re.compile(r"partition[23]_kernel|combine3_kernel|iota_kernel|red_iota_payload_kernel"),
    "replay": re.compile(r"\bingest_kernel"),
    "push_rl": re.compile(r"sp_(range|hist|scan|scatter)_kernel"),
    "fire_rl": re.compile(r"sp_(refine|agg)_kernel"),
    "fire": re.compile(r"fire_kernel|fire_multi_kernel|fire_slide_kernel|sess2_fire_kernel"),
    "sessions": re.compile(r"sess2_(?!fire)|sess3_|s4_|s5_|DeviceRadixSort|DeviceScan|radix|onesweep|lookback", re.I),
}
# the first kernel of every step of each config: counts steps in dispatch order
STEP_MARK = {"ingest": re.compile(r"partition[23]_kernel"), "push_rl": re.compile(r"sp_hist_kernel"),
             "sessions": re.compile(r"s5_hist_kernel|s4_route_kernel|sess3_min_kernel|sess2_classify_kernel")}


def load(path):
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["_t0"] = int(r["Start_Timestamp"])
        r["_t1"] = int(r["End_Timestamp"])
        r["_id"] = int(r.get("Dispatch_Id", 0) or 0)
    rows.sort(key=lambda r: r["_t0"])
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("--out")
    args = ap.parse_args()
    line = [ln for ln in open(args.bench) if ln.startswith("{")][-1]
    b = json.loads(line)
    W, K = b["warmup"], b["steps"]
    rl = b["roofline"]
    peak = rl["peak"]
    rows = load(args.trace)
    kern = rl.get("kernel", "")
    fam = "sessions" if ("sess" in kern or "s4_" in kern or "s5_" in kern) else ("push_rl" if "sp_range" in kern else "ingest")
    mark = STEP_MARK[fam]
    firsts = [r for r in rows if mark.search(r["Kernel_Name"])]
    if len(firsts) < W + K:
        sys.exit("trace has %d step marks, need warmup %d + steps %d" % (len(firsts), W, K))
    stream = firsts[0].get("Stream_Id")
    main_rows = [r for r in rows if r.get("Stream_Id") == stream] if stream is not None else rows
    marks = [r for r in main_rows if mark.search(r["Kernel_Name"])]
    # step s spans [mark s, mark s+1) on the main stream; the last timed step ends at the next mark or trace end
    t_lo = marks[W]["_t0"]
    t_hi = marks[W + K]["_t0"] if len(marks) > W + K else float("inf")
    timed = [r for r in main_rows if t_lo <= r["_t0"] < t_hi]
    out = {"trace": args.trace, "bench": args.bench, "warmup": W, "steps": K, "family": fam,
           "main_stream": stream, "timed_dispatches": len(timed), "per_kernel": {}}
    per = {}
    for r in timed:
        nm = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
        short = re.match(r"(?:void )?([A-Za-z_0-9:]+)", nm).group(1).split("::")[-1]
        per.setdefault(short, []).append((r["_t1"] - r["_t0"]) / 1e6)   # ns -> ms
    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        out["per_kernel"][k] = {"calls": len(v), "total_ms": sum(v), "avg_ms": statistics.mean(v),
                                "min_ms": min(v), "max_ms": max(v)}
    def fam_ms(f):
        return sum((r["_t1"] - r["_t0"]) / 1e6 for r in timed if FAMILIES[f].search(r["Kernel_Name"]))
    dom = fam_ms(fam)
    if fam == "ingest":
        dom_launch = dom / K
        alg = rl["alg_bytes_per_launch"]
    elif fam == "push_rl":
        dom_launch = dom / K
        alg = rl["alg_bytes_per_launch"]
    else:
        dom_launch = dom / K
        alg = rl["alg_bytes_per_launch"]
    achieved = alg / (dom_launch / 1e3) / 1e9
    out["dominant"] = {"family": fam, "ms_per_launch": dom_launch, "alg_bytes_per_launch": alg,
                       "achieved_GBps": achieved, "peak_GBps": peak, "frac": achieved / peak,
                       "bench_frac": rl["frac"], "bench_avg_launch_ms": rl.get("avg_launch_ms"),
                       "agreement": (achieved / peak) / rl["frac"] if rl["frac"] else None}
    if "roofline_fire" in b:
        rf = b["roofline_fire"]
        f_ms = fam_ms("fire_rl" if fam == "push_rl" else "fire") / K
        fa = rf["alg_bytes_per_launch"] / (f_ms / 1e3) / 1e9 if f_ms > 0 else 0.0
        out["fire"] = {"ms_per_step": f_ms, "alg_bytes_per_step": rf["alg_bytes_per_launch"], "achieved_GBps": fa,
                       "frac": fa / peak, "bench_frac": rf["frac"],
                       "agreement": (fa / peak) / rf["frac"] if rf["frac"] else None}
    step_ms = (timed[-1]["_t1"] - t_lo) / 1e6 / K if timed else 0.0
    busy = sum((r["_t1"] - r["_t0"]) / 1e6 for r in timed) / K
    out["step"] = {"span_ms_per_step_under_trace": step_ms, "gpu_busy_ms_per_step": busy,
                   "bench_ms_per_step": b["ms_per_step"]}
    js = json.dumps(out, indent=1)
    print(js)
    if args.out:
        open(args.out, "w").write(js + "\n")


if __name__ == "__main__":
    main()
