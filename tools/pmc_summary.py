"""Summarise tools/gpu_pmc_all.sh output into profiles/<tag>_pmc_<cfg>.json.

Per kernel: FETCH_SIZE and WRITE_SIZE per dispatch, as reported. MI355X_MICROARCH.md (HBM section) calibrates
FETCH_SIZE only for wide coalesced streaming reads (16 B per lane), where it reports exactly half the bytes; other
access widths are uncalibrated. So the per-step traffic is given three ways:
  raw       FETCH_SIZE + WRITE_SIZE as reported (lower bound),
  estimate  FETCH_SIZE x2 only for the kernels in WIDE (their bulk reads are 16 B/lane streaming loads,
            as noted at WIDE) + WRITE_SIZE -- this is `ingest_bytes_per_launch`, the bench's `traffic`,
  upper     FETCH_SIZE x2 for every kernel + WRITE_SIZE (upper bound).
Per timed step: the ingest kernels (everything but the fire, generator, torch and runtime-copy kernels) over the
last `steps` steps' dispatches, against the algorithmic bytes of the step (24 B per record, 28 B
for the C5 float columns).
"""
import csv
import glob
import json
import os
import re
import sys

EXCLUDE = re.compile(r"fire|sp_refine|sp_agg|generate_kernel|reduce_kernel|elementwise|rocclr|reset|fill_u64|push_reset|wire_")
FIRE = re.compile(r"fire|sp_agg")   # one per step: marks the timed region
# kernels whose bulk reads are 16 B-per-lane coalesced streaming loads (the calibrated case)
WIDE = {
    "partition3_kernel",   # engine.hip load_pairs: ulonglong2 / longlong2 key, ts, value loads
    "sp_agg_kernel",       # sparse.inc: 16-byte entry loads over contiguous bucket runs
    "wire_scan_kernel",    # wire.hip: 16-byte chunk loads
    "wire_decode_kernel",
}


def short(name):
    m = re.search(r"(?:::)?([A-Za-z_][A-Za-z0-9_]*)(?:<|\()", name)
    base = m.group(1) if m else name[:40]
    if "DeviceRadixSort" in name or "radix" in name.lower():
        base = "hipcub_radix_sort"
    elif "DeviceScan" in name or "scan" in name.lower() and "hipcub" in name.lower():
        base = "hipcub_scan"
    return base


def read(path):
    f = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return {}
    per = {}
    with open(f[0]) as fh:
        for r in csv.DictReader(fh):
            k = short(r["Kernel_Name"])
            per.setdefault(k, []).append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    for k in per:
        per[k].sort()
    return per


def main(root, tag, steps=3):
    out_dir = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")
    for cfg in ("c2", "c3", "c4", "c5", "c5s", "reduce"):
        fe = read(os.path.join(root, "%s_FETCH_SIZE" % cfg))
        wr = read(os.path.join(root, "%s_WRITE_SIZE" % cfg))
        if not fe or not wr:
            continue
        warm = 2 if cfg == "c3" else 1
        total_steps = steps + warm
        # timed steps = the dispatches after the last warm-up step's fire (one fire kernel per step)
        fires = sorted(d for k, v in fe.items() if FIRE.search(k) for d, _ in v)
        bound = fires[len(fires) - steps - 1] if len(fires) > steps else -1
        res = {}
        tot = {"raw": 0.0, "estimate": 0.0, "upper": 0.0}
        for k in sorted(set(fe) | set(wr)):
            f = [(d, v * 1024) for d, v in fe.get(k, [])]   # KB -> bytes, as reported
            w = [(d, v * 1024) for d, v in wr.get(k, [])]
            res[k] = {"dispatches": max(len(f), len(w)), "fetch_bytes_raw_per_dispatch": [v for _, v in f],
                      "write_bytes_per_dispatch": [v for _, v in w], "wide_streaming_reads": k in WIDE}
            if not EXCLUDE.search(k):
                tf = sum(v for d, v in f if d > bound) / steps
                tw = sum(v for d, v in w if d > bound) / steps
                b = {"raw": tf + tw, "estimate": tf * (2 if k in WIDE else 1) + tw, "upper": 2 * tf + tw}
                res[k]["bytes_per_timed_step"] = b
                res[k]["timed_dispatches"] = len([1 for d, _ in f if d > bound])
                for x in tot:
                    tot[x] += b[x]
        step_bytes = tot["estimate"]
        batch = 1 << 26
        rec = 28 if cfg in ("c5", "c5s") else 24
        doc = {"note": "rocprofv3 --pmc FETCH_SIZE; WRITE_SIZE in separate runs (tools/gpu_pmc_all.sh), bench.py "
                       "--config %s --steps %d --warmup %d; FETCH_SIZE x2 only for the WIDE kernels (gfx950 calibration), "
                       "WRITE_SIZE as reported; raw and upper bounds beside the estimate; "
                       "ingest = every kernel except fire (incl. the record-list refine / aggregate) / generator / torch / runtime copies, dispatched after the warm-up's last fire (%d timed steps)"
                       % (cfg, steps, warm, steps),
               "config": {"workload": cfg, "batch": batch}, "per_kernel": res,
               "wide_kernels": sorted(WIDE), "ingest_bytes_per_launch": step_bytes,
               "ingest_bytes_per_launch_bounds": {"raw": tot["raw"], "upper": tot["upper"]},
               "alg_bytes_per_launch": rec * batch, "traffic_over_alg": step_bytes / (rec * batch),
               "traffic_over_alg_bounds": {"raw": tot["raw"] / (rec * batch), "upper": tot["upper"] / (rec * batch)}}
        with open(os.path.join(out_dir, "%s_pmc_%s.json" % (tag, cfg)), "w") as fh:
            json.dump(doc, fh, indent=1)
        print(cfg, "ingest bytes/step %.3g" % step_bytes, "x alg %.2f (raw %.2f, upper %.2f)"
              % (step_bytes / (rec * batch), tot["raw"] / (rec * batch), tot["upper"] / (rec * batch)),
              {k: round(v["bytes_per_timed_step"]["estimate"] / 1e6) for k, v in res.items() if "bytes_per_timed_step" in v})


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmca", sys.argv[2] if len(sys.argv) > 2 else "r03")
