"""Per-step cost of the N>1 two-phase plan's pieces on one GPU (C2 batch): local push, drain_partials, GPU routing
(fwa_route_rows, world 8), owner push_partials of the whole drained set (the volume an owner merges per step under
weak scaling). No collective: the all_to_all is priced separately from the bytes shipped."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from flink_amd import _abi as A  # noqa: E402
from flink_amd import engine as E  # noqa: E402

B = 1 << 26
S = 4
p = A.GenParams(seed_k=1, seed_t=2, seed_v=3, first_index=0, total_records=S * B, num_keys=1_000_000,
                t0_ms=1_700_000_000_000, span_ms=S * B * 1_000_000 // 1_000_000_000, max_delay_ms=1000, key_dist=0, val_kind=0)
dev = torch.device("cuda", 0)
keys = torch.empty(S * B, dtype=torch.int64, device=dev)
ts = torch.empty_like(keys)
vals = torch.empty_like(keys)
E.generate(p, S * B, keys, ts, vals)
torch.cuda.synchronize()
kw = dict(window_kind="TUMBLE", size_ms=10_000, aggs=[("COUNT", 0), ("SUM_I64", 0)], key_capacity=1_000_000,
          output_on_device=1)
local = E.WindowAggregator(A.make_config(**kw))
owner = E.WindowAggregator(A.make_config(**kw))
m = -2**63
for b in range(S):
    sl = slice(b * B, (b + 1) * B)
    m = max(m, int(ts[sl].max().item()))
    wm = m - 1001
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    local.push(keys[sl], ts[sl], [vals[sl]])
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    d = local.drain_partials(wm)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    cols = [d["key"], d["slice_start"], d["count"]] + [d["acc%d" % j] for j in range(2)]
    packed, counts = E.route_rows(cols[0], cols, 128, 8)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    c = E.unpack_rows(packed)
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    owner.push_partials(c[0], c[1], c[2], c[3:])
    torch.cuda.synchronize()
    t5 = time.perf_counter()
    n = owner.advance_watermark_raw(wm).n_rows
    torch.cuda.synchronize()
    t6 = time.perf_counter()
    print("step %d: push %.3f drain %.3f route %.3f unpack %.3f push_partials %.3f fire %.3f ms; partials %d (%.0f MB), rows %d"
          % (b, (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t4 - t3) * 1e3, (t5 - t4) * 1e3, (t6 - t5) * 1e3,
             d["key"].shape[0], packed.numel() * 8 / 1e6, n), flush=True)
