import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from flink_amd import _abi as A
from flink_amd import engine as E
d = np.load(sys.argv[1])
keys, ts = d["keys"], d["ts"]
cfg = A.make_config(window_kind="SESSION", gap_ms=600, aggs=[("COUNT", 0)], key_capacity=4096)
g = E.WindowAggregator(cfg)
g.push(keys, ts, [keys])
r = g.advance_watermark(A.LONG_MAX)
print("rows", len(r["key"]), r["key"][:5], r["win_start"][:5], r["win_end"][:5], r["agg0"][:5])
