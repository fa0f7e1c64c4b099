"""Per-rank step of the N>1 raw-record keyBy plan (C4: 1e8 keys, record lists) on one GPU, against the N=1 step.

Weak scaling at N = WORLD: every rank routes its own 2^26 records by key group (fwa_route_rows: a GPU counting sort into
packed int64 rows, one block per destination), ships WORLD-1 of the blocks over xGMI and receives as many records from
the others -- with uniform keys one 2^26-record batch of its own key groups' records -- which its owner engine unpacks
and pushes, then fires. Priced here on one MI355X: the route of a batch, the unpack of 2^26 received rows, the owner's
push of them and its fire (the owner holds 1/WORLD of the key groups; record-list key spaces keep their full key
capacity). The all-to-all is a model (it needs WORLD GPUs): the bytes sent to each peer / the per-link xGMI rate
(--link-gbps, SURVEY.md section 5: ~153 GB/s per link and direction, one link per peer, all links in parallel) /
--link-eff; "narrow" prices rows of 12 bytes (32-bit key, 32-bit value, 32-bit timestamp offset) instead of 24, the
compressed variant the model asks about. Output: tools/raw_cost.py > profiles/<tag>_raw_cost.txt."""
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
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--keys", type=int, default=100_000_000)
ap.add_argument("--link-gbps", type=float, default=153.0)
ap.add_argument("--link-eff", type=float, default=0.8)
args = ap.parse_args()

B = 1 << 26
S = args.steps
W = args.world
p = A.GenParams(seed_k=1, seed_t=2, seed_v=3, first_index=0, total_records=S * B, num_keys=args.keys,
                t0_ms=1_700_000_000_000, span_ms=S * B * 1_000_000 // 1_000_000_000, max_delay_ms=1000, key_dist=0,
                val_kind=0)
dev = torch.device("cuda", 0)
keys = torch.empty(S * B, dtype=torch.int64, device=dev)
ts = torch.empty_like(keys)
vals = torch.empty_like(keys)
E.generate(p, S * B, keys, ts, vals)
torch.cuda.synchronize()
bmax = ts.view(S, B).max(dim=1).values.cpu().tolist()
kw = dict(window_kind="TUMBLE", size_ms=10_000, aggs=[("COUNT", 0), ("SUM_I64", 0)], key_capacity=args.keys,
          output_on_device=1)
single = E.WindowAggregator(A.make_config(**kw))
kg0, kg1 = key_group_range_for_operator(128, W, 0)
owner = E.WindowAggregator(A.make_config(kg_start=kg0, kg_end=kg1, **kw))
print("world %d, owner key groups [%d, %d], record lists %s" % (W, kg0, kg1, owner.record_lists), flush=True)


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    return r, (time.perf_counter() - t0) * 1e3


# the owner's receive buffer: this rank's own records of the owner's key groups, as many as WORLD sources send
_, op_all = E.key_groups(keys, 128, W)
own = torch.as_tensor(op_all, device=dev) == 0 if not isinstance(op_all, torch.Tensor) else op_all.to(dev) == 0
m = -2**63
tot = {}
for b in range(S):
    sl = slice(b * B, (b + 1) * B)
    m = max(m, int(bmax[b]))
    wm = m - 1001
    t = {}
    _, t["n1_push"] = timed(lambda: single.push(keys[sl], ts[sl], [vals[sl]]))
    _, t["n1_fire"] = timed(lambda: single.advance_watermark_raw(wm).n_rows)
    (packed, counts), t["route"] = timed(lambda: E.route_rows(keys[sl], [keys[sl], ts[sl], vals[sl]], 128, W))
    peer_rows = int(counts[1:].max().item())
    # received: the owner's key groups from every source = about one batch; take this rank's share W times over the
    # stream window around the batch (the same event-time range), as the W sources would send it
    sel = own[b * B:(b + 1) * B]
    rk, rt, rv = keys[sl][sel], ts[sl][sel], vals[sl][sel]
    recv = torch.stack([rk, rt, rv], 1).repeat(W, 1)
    c, t["unpack"] = timed(lambda: E.unpack_rows(recv))
    _, t["owner_push"] = timed(lambda: owner.push(c[0], c[1], [c[2]]))
    _, t["owner_fire"] = timed(lambda: owner.advance_watermark_raw(wm).n_rows)
    if b >= 1:
        for k, v in t.items():
            tot[k] = tot.get(k, 0.0) + v
        tot["peer_rows"] = tot.get("peer_rows", 0) + peer_rows
    print("step %d: " % b + " ".join("%s %.3f" % kv for kv in t.items()) + " ms; rows to each peer %d" % peer_rows,
          flush=True)
n = S - 1
n1 = (tot["n1_push"] + tot["n1_fire"]) / n
rows = tot["peer_rows"] / n
print("N=1 step %.3f ms (push %.3f, fire %.3f)" % (n1, tot["n1_push"] / n, tot["n1_fire"] / n))
dev_ms = sum(tot[k] for k in ("route", "unpack", "owner_push", "owner_fire")) / n
print("N=%d per-rank step without the exchange: %.3f ms = route %.3f + unpack %.3f + owner push %.3f + fire %.3f "
      "-> %.2fx N=1" % (W, dev_ms, tot["route"] / n, tot["unpack"] / n, tot["owner_push"] / n, tot["owner_fire"] / n,
                        dev_ms / n1))
for name, rb in (("24-byte rows", 24), ("narrow 12-byte rows", 12)):
    x = rows * rb / (args.link_gbps * 1e9 * args.link_eff) * 1e3
    print("  all-to-all model, %s: %.1f MB to each peer at %.0f GB/s x %.2f = %.3f ms; serial step %.3f ms -> %.2fx; "
          "pipelined max(route, exchange) + owner %.3f ms -> %.2fx N=1" %
          (name, rows * rb / 1e6, args.link_gbps, args.link_eff, x, dev_ms + x, (dev_ms + x) / n1,
           max(tot["route"] / n, x) + dev_ms - tot["route"] / n, (max(tot["route"] / n, x) + dev_ms - tot["route"] / n) / n1))
