"""Debug: the bench's C4 N=2 raw loop (generator, KeyedWindowPipeline, device-output fires), counting foreign keys
after every exchange."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from flink_amd import _abi as A, engine as E  # noqa: E402
from flink_amd.distributed import KeyedWindowPipeline, exchange_rows  # noqa: E402

dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
B, S = 1 << 22, 3
n = B * S
p = A.GenParams(seed_k=0x5eed0001 ^ (rank * 0x9E3779B97F4A7C15 & 0xFFFFFFFFFFFFFFFF), seed_t=0x5eed0002 + rank,
                seed_v=0x5eed0003 + rank, first_index=0, total_records=n, num_keys=100_000_000, t0_ms=1_700_000_000_000,
                span_ms=n * 1000 // 1_000_000, max_delay_ms=1000, key_dist=0, val_kind=0)
keys = torch.empty(n, dtype=torch.int64, device=dev)
ts = torch.empty_like(keys)
vals = torch.empty_like(keys)
E.generate(p, n, keys, ts, vals, device=0)
torch.cuda.synchronize()
pipe = KeyedWindowPipeline(rank, world, window_kind="TUMBLE", semantics="DATASTREAM", size_ms=10_000,
                           aggs=[("COUNT", 0), ("SUM_I64", 0)], key_capacity=100_000_000, output_on_device=1, device=0)
lo, hi = pipe.cfg.kg_start, pipe.cfg.kg_end
m = -2**63
for b in range(S):
    k, t, v = keys[b * B:(b + 1) * B], ts[b * B:(b + 1) * B], vals[b * B:(b + 1) * B]
    recv = exchange_rows(pipe, k, [k, t, v])
    rk = recv[:, 0].contiguous()
    kg, _ = E.key_groups(rk.cpu().numpy(), 128, 1, A.KEY_JAVA_LONG)
    print("rank %d batch %d recv %d foreign %d" % (rank, b, len(kg), int(((kg < lo) | (kg > hi)).sum())), flush=True)
    try:
        pipe.engine.push(rk, recv[:, 1].contiguous(), [recv[:, 2].contiguous()])
        print("rank %d batch %d push ok" % (rank, b), flush=True)
    except Exception as ex:
        print("rank %d batch %d push failed: %s" % (rank, b, ex), flush=True)
        break
    m = max(m, int(t.max()))
    r = pipe.advance_watermark(m - 1001, device_output=True)
    print("rank %d batch %d fired %d" % (rank, b, int(r["key"].shape[0])), flush=True)
pipe.close()
dist.destroy_process_group()
