"""Child-process parity check with the adaptive combiner modes forced on from the first push (fwa_set_option
FWA_OPT_SKEW_MERGE = 1: Phase P tile pre-aggregation, FWA_OPT_WINDOW_PASSES = 1: window passes), so random streams
exercise them at small sizes. Run by tests/test_skew_gpu.py::test_forced_pre_and_window_passes; exits non-zero on a
mismatch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from flink_amd import _abi as A  # noqa: E402
from flink_amd import engine  # noqa: E402
from helpers import assert_rows_equal  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

CONFIGS = [
    dict(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=1000),
    dict(window_kind="SLIDE", semantics="TABLE", size_ms=4000, slide_ms=250),
    dict(window_kind="CUMULATE", semantics="TABLE", size_ms=3000, slide_ms=200),
    dict(window_kind="SLIDE", semantics="DATASTREAM", size_ms=3000, slide_ms=500, allowed_lateness_ms=700),
]
AGGS = [[("COUNT", 0), ("SUM_I64", 0)], [("COUNT", 0)], [("COUNT", 0), ("SUM_F64", 1), ("MAX_F64", 1)]]


def main():
    engine.DEFAULT_OPTIONS.update(skew_merge=1, window_passes=1)   # every handle of this process
    for ci, kw in enumerate(CONFIGS):
        for ai, aggs in enumerate(AGGS):
            rng = np.random.default_rng(100 * ci + ai)
            n, nkeys, delay = 120_000, 3000, 1500
            keys = rng.zipf(1.3, n).astype(np.int64) % nkeys
            ts = np.sort(rng.integers(0, 90_000, n)).astype(np.int64) - rng.integers(0, delay + 1, n)
            late = rng.random(n) < 0.02
            ts[late] -= rng.integers(delay, 4 * delay, late.sum())
            vi = rng.integers(-2**40, 2**40, n).astype(np.int64)
            vd = rng.random(n) * 100.0
            cfg = A.make_config(aggs=aggs, key_capacity=1 << 14, **kw)
            names = A.agg_names(cfg)
            g, o = engine.WindowAggregator(cfg), Oracle(cfg)
            mx, nb = -2**63, 8
            for b in range(nb + 1):
                sl = slice(b * n // nb, (b + 1) * n // nb) if b < nb else slice(0, 0)
                cols = [vi[sl], vd[sl]]
                assert g.push(keys[sl], ts[sl], cols) == o.push(keys[sl], ts[sl], cols)
                if b < nb:
                    mx = max(mx, int(ts[sl].max()))
                wm = mx - delay - 1 if b < nb else A.LONG_MAX
                assert_rows_equal(g.advance_watermark(wm), o.advance_watermark(wm), names, rtol=1e-9,
                                  ctx="config %d aggs %d wm=%d" % (ci, ai, wm))
            g.close()
            o.close()
    print("forced modes ok")


if __name__ == "__main__":
    main()
