"""Per-rank step cost of the N>1 two-phase plan on one GPU (C2 batch), against the N=1 step (push + fire).

Each step prices the pieces one rank runs at N = WORLD (default 8) under weak scaling:
  local  push (the rank's own 2^26 records), then fwa_drain_route (drain + routing by key group, WORLD ways, in one
         pass; --routed 0: drain_partials, then fwa_route_rows);
  owner  what it does with what it receives -- this rank's rows for destination 0, repeated WORLD times (one copy
         per source rank: the same keys and windows, each source holding its own partial), sources back to back as
         in the receive buffer: "merge_fire" = fwa_fire_partials on the packed rows (the pipeline's path), "sources"
         = unpack + push_partials + fire, "window" = the same with the rows sorted window-major first.
The all_to_all is priced by a model (it needs W GPUs): bytes this rank sends to each peer / the per-link xGMI rate
(--link-gbps, default SURVEY.md section 5's ~153 GB/s per link and direction, one link per peer in an 8-GPU mesh, all
links in parallel) / --link-eff; the step is printed serial (exchange added) and pipelined (bench.py overlaps the
exchange with the next batch's push: max(local, exchange) + owner). The owner engine is sized to its key-group share
(distributed.owner_key_capacity)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from flink_amd import _abi as A  # noqa: E402
from flink_amd import engine as E  # noqa: E402
from flink_amd.keygroups import key_group_range_for_operator  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--steps", type=int, default=6)
ap.add_argument("--order", default="merge_fire,sources")
ap.add_argument("--owner-share", type=int, default=1, help="1: owner key capacity sized to its key-group share")
ap.add_argument("--dup", type=int, default=0, help="copies of the destination-0 rows the owner receives (0: world)")
ap.add_argument("--routed", type=int, default=1, help="1: fwa_drain_route (drain + routing in one pass)")
ap.add_argument("--owner-profile", type=int, default=0, help="FWA_OPT_PROFILE on the owners (per-block phase cycles)")
ap.add_argument("--link-gbps", type=float, default=153.0, help="assumed xGMI rate per link and direction (GB/s)")
ap.add_argument("--link-eff", type=float, default=0.8, help="assumed all-to-all efficiency on those links")
args = ap.parse_args()

B = 1 << 26
S = args.steps
W = args.world
KEYS = 1_000_000
p = A.GenParams(seed_k=1, seed_t=2, seed_v=3, first_index=0, total_records=S * B, num_keys=KEYS,
                t0_ms=1_700_000_000_000, span_ms=S * B * 1_000_000 // 1_000_000_000, max_delay_ms=1000, key_dist=0,
                val_kind=0)
dev = torch.device("cuda", 0)
keys = torch.empty(S * B, dtype=torch.int64, device=dev)
ts = torch.empty_like(keys)
vals = torch.empty_like(keys)
E.generate(p, S * B, keys, ts, vals)
torch.cuda.synchronize()
bmax = ts.view(S, B).max(dim=1).values.cpu().tolist()
kw = dict(window_kind="TUMBLE", size_ms=10_000, aggs=[("COUNT", 0), ("SUM_I64", 0)], key_capacity=KEYS,
          output_on_device=1)
single = E.WindowAggregator(A.make_config(**kw))
local = E.WindowAggregator(A.make_config(**kw))
kg0, kg1 = key_group_range_for_operator(128, W, 0)
okw = dict(kw)
if args.owner_share:
    from flink_amd.distributed import owner_key_capacity
    okw["key_capacity"] = owner_key_capacity(KEYS, kg1 - kg0 + 1, 128)
orders = args.order.split(",")
owners = {o: E.WindowAggregator(A.make_config(kg_start=kg0, kg_end=kg1, **okw)) for o in orders}
for o in owners.values():
    if args.owner_profile:
        o.set_option("profile", 1)
print("world %d, owner key groups [%d, %d], owner key capacity %d" % (W, kg0, kg1, okw["key_capacity"]), flush=True)


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    return r, (time.perf_counter() - t0) * 1e3


m = -2**63
tot = {}
for b in range(S):
    sl = slice(b * B, (b + 1) * B)
    m = max(m, int(bmax[b]))
    wm = m - 1001
    t = {}
    _, t["n1_push"] = timed(lambda: single.push(keys[sl], ts[sl], [vals[sl]]))
    _, t["n1_fire"] = timed(lambda: single.advance_watermark_raw(wm).n_rows)
    _, t["push"] = timed(lambda: local.push(keys[sl], ts[sl], [vals[sl]]))
    if args.routed:     # fwa_drain_route: the drain writes the per-destination send blocks itself
        (parts, counts, m), t["drain_route"] = timed(lambda: local.drain_route(wm, W))
        peer_bytes = max(counts[1:]) * m * 8 if W > 1 else 0
        recv = parts[0].repeat(args.dup or W, 1)
        d = {"key": torch.empty(sum(counts))}
        packed = torch.empty((sum(counts), m), dtype=torch.int64)
    else:
        d, t["drain"] = timed(lambda: local.drain_partials(wm))
        cols = [d["key"], d["slice_start"], d["count"], d["acc1"]]
        (packed, counts), t["route"] = timed(lambda: E.route_rows(cols[0], cols, 128, W))
        n0 = int(counts[0].item())
        peer_bytes = int(counts[1:].max().item()) * len(cols) * 8 if W > 1 else 0
        recv = packed[:n0].repeat(args.dup or W, 1)                 # what the owner receives: one copy per source rank
    cells = [2, 3]
    for o in orders:
        if o == "merge_fire":
            _, t[o] = timed(lambda: owners[o].fire_partials(recv, cells, wm, device_output=True)["key"].shape[0])
            continue
        rv = recv
        if o == "window":                               # window-major: all sources' rows of a window together
            rv = recv[torch.argsort(recv[:, 1], stable=True)]
        c, t[o + "_unpack"] = timed(lambda: E.unpack_rows(rv))
        _, t[o + "_merge"] = timed(lambda: owners[o].push_partials(c[0], c[1], c[2], [c[2], c[3]]))
        _, t[o + "_fire"] = timed(lambda: owners[o].advance_watermark_raw(wm).n_rows)
    xm = peer_bytes / (args.link_gbps * 1e9 * args.link_eff) * 1e3
    if b >= 2:
        for k, v in t.items():
            tot[k] = tot.get(k, 0.0) + v
        tot["exchange_model"] = tot.get("exchange_model", 0.0) + xm
        tot["peer_mb"] = tot.get("peer_mb", 0.0) + peer_bytes / 1e6
    print("step %d: " % b + " ".join("%s %.3f" % kv for kv in t.items()) +
          " ms; partials %d (%.0f MB), owner rows %d" % (d["key"].shape[0], packed.numel() * 8 / 1e6, recv.shape[0]),
          flush=True)
n = S - 2
n1 = (tot["n1_push"] + tot["n1_fire"]) / n
print("N=1 step %.3f ms (push %.3f, fire %.3f)" % (n1, tot["n1_push"] / n, tot["n1_fire"] / n))
for o in orders:
    parts = ["push"] + (["drain_route"] if args.routed else ["drain", "route"]) + \
        ([o] if o == "merge_fire" else [o + "_unpack", o + "_merge", o + "_fire"])
    s = sum(tot[k] for k in parts) / n
    print("N=%d per-rank step, owner order %s: %.3f ms = %s -> %.2fx N=1" %
          (W, o, s, " + ".join("%s %.3f" % (k, tot[k] / n) for k in parts), s / n1))
    x = tot["exchange_model"] / n
    local = sum(tot[k] for k in parts[:2 if args.routed else 3]) / n
    owner = s - local
    print("  with the all-to-all (model: %.1f MB to each peer at %.0f GB/s x %.2f = %.3f ms): serial %.3f ms -> %.2fx; "
          "pipelined max(local %.3f, exchange) + owner %.3f = %.3f ms -> %.2fx N=1" %
          (tot["peer_mb"] / n, args.link_gbps, args.link_eff, x, s + x, (s + x) / n1, local, owner,
           max(local, x) + owner, (max(local, x) + owner) / n1))
