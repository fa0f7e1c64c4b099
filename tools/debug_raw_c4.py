"""Debug: 2 ranks (gloo, one GPU) -- route C4-like keys with fwa_route_rows, exchange, and count received keys whose
key group this rank does not own; then push them into a record-list engine owning the rank's range."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from flink_amd import _abi as A, engine as E  # noqa: E402
from flink_amd.distributed import KeyedWindowPipeline, exchange_rows  # noqa: E402
from flink_amd.keygroups import key_group_range_for_operator  # noqa: E402

dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
torch.cuda.set_device(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
rng = np.random.default_rng(rank)
keys = torch.from_numpy(rng.integers(0, 100_000_000, n).astype(np.int64)).cuda()
ts = torch.from_numpy(np.sort(rng.integers(0, 60_000, n)).astype(np.int64)).cuda()
vals = torch.from_numpy(rng.integers(0, 100, n).astype(np.int64)).cuda()
for cap in (1_000_000, 100_000_000):
    pipe = KeyedWindowPipeline(rank, world, window_kind="TUMBLE", semantics="DATASTREAM", size_ms=10_000,
                               aggs=[("COUNT", 0), ("SUM_I64", 0)], key_capacity=cap)
    recv = exchange_rows(pipe, keys, [keys, ts, vals])
    k = recv[:, 0].contiguous().cpu().numpy()
    kg, _ = E.key_groups(k, 128, 1, A.KEY_JAVA_LONG)
    lo, hi = key_group_range_for_operator(128, world, rank)
    bad = int(((kg < lo) | (kg > hi)).sum())
    print("rank %d cap %d recv %d foreign %d range [%d,%d] cfg kg [%d,%d] rl %d" % (
        rank, cap, len(k), bad, lo, hi, pipe.cfg.kg_start, pipe.cfg.kg_end, pipe.engine.record_lists), flush=True)
    try:
        pipe.push(keys, ts, [vals])
        print("rank %d cap %d push ok" % (rank, cap), flush=True)
    except Exception as ex:
        print("rank %d cap %d push failed: %s" % (rank, cap, ex), flush=True)
    pipe.close()
dist.destroy_process_group()
