"""Find a small failing input for the sessions cell path (one push, fire everything) and print the differing rows."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from flink_amd import _abi as A
from flink_amd import engine as E
from oracle.oracle import Oracle

def rows(d):
    return sorted(zip(*[list(map(int, d[k])) for k in ("key", "win_start", "win_end", "agg0")]))

def run(keys, ts, gap):
    cfg = A.make_config(window_kind="SESSION", gap_ms=gap, aggs=[("COUNT", 0)], key_capacity=4096)
    g = E.WindowAggregator(cfg); o = Oracle(cfg)
    g.push(keys, ts, [keys]); o.push(keys, ts, [keys])
    a = g.advance_watermark(A.LONG_MAX); b = o.advance_watermark(A.LONG_MAX)
    g.close(); o.close()
    return rows(a), rows(b)

rng = np.random.default_rng(7)
for nk in (1, 2, 3, 5, 10, 50, 700):
    for trial in range(20):
        n = int(rng.integers(50, 4000))
        keys = rng.integers(0, nk, n).astype(np.int64)
        ts = np.sort(rng.integers(0, 5000, n)).astype(np.int64) - rng.integers(0, 1200, n)
        ra, rb = run(keys, ts, 600)
        if ra != rb:
            print("FAIL nk", nk, "n", n, "rows", len(ra), len(rb))
            sa, sb = set(ra), set(rb)
            print("engine only:", sorted(sa - sb)[:12])
            print("oracle only:", sorted(sb - sa)[:12])
            np.savez("gpurun_out/dbg_cell_case.npz", keys=keys, ts=ts)
            sys.exit(0)
print("no failure found")
