"""Full-size parity of the benched configurations: every fired row, not only totals.

The C2 stream bench.py times (15 batches of 2^26 records, 1M uniform keys, tumbling 10 s COUNT + SUM(long), D = 1 s,
async device pushes, output left in HBM) and the C4 one (1e8 uniform keys, record lists auto-selected; 5 batches of
2^26 records at the bench's event-time density, to bound the oracle's time) go through the engine; per watermark the
fired rows' count and order-free digest (tests/digest.py, computed with torch on the device columns) must equal those
of the threaded oracle (or_pipeline_digests: one WindowOperator restatement per key-group range over the same
generated stream, WindowOperator.onEventTime, WindowOperator.java:437-481). The oracle runs in a thread beside the GPU
run (ctypes releases the GIL)."""
import os
import threading

import numpy as np
import pytest

from digest import rows_digest
from flink_amd import _abi as A

pytestmark = pytest.mark.gpu

B = 1 << 26


def _threads():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(q) // int(period)))
    except (OSError, ValueError):
        pass
    return max(1, min(n, 32))


def _digest_run(nkeys, nbatches, record_lists):
    import torch
    from flink_amd import engine as E
    from oracle import oracle as O
    n = nbatches * B
    p = A.GenParams(seed_k=0x5eed0001, seed_t=0x5eed0002, seed_v=0x5eed0003, first_index=0, total_records=n,
                    num_keys=nkeys, t0_ms=1_700_000_000_000, span_ms=n * 1_000_000 // 1_000_000_000,
                    max_delay_ms=1000, key_dist=0, val_kind=0)
    ocfg = A.make_config(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=10_000,
                         aggs=[("COUNT", 0), ("SUM_I64", 0)])
    res = {}

    def oracle_leg():
        try:
            res["oracle"] = O.pipeline_digests(ocfg, p, n, B, _threads())
        except Exception as ex:      # reported by the main thread
            res["error"] = ex
    th = threading.Thread(target=oracle_leg)
    th.start()
    try:
        k = torch.empty(n, dtype=torch.int64, device="cuda")
        t = torch.empty_like(k)
        v = torch.empty_like(k)
        E.generate(p, n, k, t, v)
        torch.cuda.synchronize()
        bmax = t.view(nbatches, B).max(dim=1).values.cpu().numpy()
        cfg = A.make_config(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=10_000,
                            aggs=[("COUNT", 0), ("SUM_I64", 0)], key_capacity=nkeys, output_on_device=1)
        g = E.WindowAggregator(cfg)
        assert g.record_lists == record_lists
        got = []
        m = -2**63
        for b in range(nbatches + 1):
            if b < nbatches:
                m = max(m, int(bmax[b]))
                g.push(k[b * B:(b + 1) * B], t[b * B:(b + 1) * B], [v[b * B:(b + 1) * B]], sync=False)
                wm = m - 1001
            else:
                wm = A.LONG_MAX
            out = g.advance_watermark_device(wm)
            got.append(rows_digest(out["key"], out["win_start"], out["win_end"], [out["agg0"], out["agg1"]]))
        st = g.stats()
        assert st.records_in == n and st.late_dropped == 0
        g.close()
        del k, t, v
    finally:
        th.join()
    if "error" in res:
        raise res["error"]
    _, rows, dig = res["oracle"]
    exp = [(int(rows[b]), int(dig[b])) for b in range(nbatches + 1)]
    assert sum(r for r, _ in got) == sum(r for r, _ in exp), (got, exp)
    for b in range(nbatches + 1):
        assert got[b] == exp[b], "watermark %d: GPU (rows, digest) %s != oracle %s" % (b, got[b], exp[b])
    return sum(r for r, _ in got)


def test_c2_full_size_rows_vs_oracle():
    """BASELINE C2 as benched: 15 x 2^26 = 1.007e9 records, 1M keys; every (key, window) row of every watermark."""
    rows = _digest_run(1_000_000, 15, record_lists=False)
    assert rows > 90_000_000                     # ~1M keys x ~100 windows


def test_c4_full_size_rows_vs_oracle():
    """BASELINE C4 engine shape at N=1: 1e8 keys (record lists), 5 x 2^26 records; every row of every watermark."""
    rows = _digest_run(100_000_000, 5, record_lists=True)
    assert rows > 200_000_000
