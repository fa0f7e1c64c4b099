"""Parity at the exact kernel instantiations bench.py times (VERDICT r1 weak #1a/#1b) and full-size
property checks of the benched configurations.

* C5 as benched: COUNT, SUM(d), AVG(d), MAX(f), MAX(d) over a FLOAT column 0 and a DOUBLE column 1
  (two carried value columns of different widths, shared SUM/AVG accumulator, generic combiner layout,
  adaptive segment size), Table TUMBLE with and without offset, against the oracle.
* C4 as benched: a key table larger than 2^22 slots (the single-pass ingest is the primary path) over a
  1e8-key uniform stream, maxParallelism 128, whole and partial key-group ranges, against the oracle.
* Full size: the C2 and C4 bench workloads (15 batches of 2^26 records, async pushes, device-resident
  output) with conservation of COUNT and SUM(long) over every fired row -- COUNT sum + late drops equals
  the record count and the SUM column totals the value column (int64 wrap-around arithmetic).

Tolerances: SUM/AVG over DOUBLE 1e-9 relative (reordering of <= 1e4 additions of [0, 1) values, the
GPU sums in a different order than the reference's sequential loop); MAX is exact.
"""
import numpy as np
import pytest

from flink_amd import _abi as A
from helpers import assert_rows_equal

pytestmark = pytest.mark.gpu

C5_AGGS = [("COUNT", 0), ("SUM_F64", 1), ("AVG_F64", 1), ("MAX_F32", 0), ("MAX_F64", 1)]
TOL = {"SUM_F64": 1e-9, "AVG_F64": 1e-9}


def _gen(eng_mod, n, nkeys, seed, val_kind, span_ms, delay=1000, first=0, total=None):
    import torch
    p = A.GenParams(seed_k=seed, seed_t=seed + 1, seed_v=seed + 2, first_index=first,
                    total_records=total or n, num_keys=nkeys, t0_ms=1_700_000_000_000, span_ms=span_ms,
                    max_delay_ms=delay, key_dist=0, val_kind=val_kind)
    k = torch.empty(n, dtype=torch.int64, device="cuda")
    t = torch.empty_like(k)
    if val_kind == 1:
        vf = torch.empty(n, dtype=torch.float32, device="cuda")
        vd = torch.empty(n, dtype=torch.float64, device="cuda")
        eng_mod.generate(p, n, k, t, None, vf, vd)
        cols = [vf, vd]
    else:
        v = torch.empty_like(k)
        eng_mod.generate(p, n, k, t, v)
        cols = [v]
    torch.cuda.synchronize()
    return k, t, cols


def _run_batches(g, o, k, t, cols, nb, delay, names, tol=None):
    kh, th = k.cpu().numpy(), t.cpu().numpy()
    ch = [c.cpu().numpy() for c in cols]
    n = kh.shape[0]
    max_ts = -2**63
    dg = do = 0
    for b in range(nb + 1):
        if b < nb:
            sl = slice(b * n // nb, (b + 1) * n // nb)
            dg += g.push(k[sl], t[sl], [c[sl] for c in cols])
            do += o.push(kh[sl], th[sl], [c[sl] for c in ch])
            max_ts = max(max_ts, int(th[sl].max()))
            wm = max_ts - delay - 1
        else:
            wm = A.LONG_MAX
        assert_rows_equal(g.advance_watermark(wm), o.advance_watermark(wm), names, rtol=tol, ctx="wm=%d" % wm)
    assert dg == do
    return dg


@pytest.fixture(scope="module")
def eng_mod():
    from flink_amd import engine
    engine.lib()
    return engine


@pytest.mark.parametrize("offset", [0, -3_700])
def test_c5_bench_aggregates_vs_oracle(eng_mod, offset):
    """bench.py --config c5 aggregate list and column layout (f32 col 0, f64 col 1), 1M-key table."""
    from oracle.oracle import Oracle
    n = 1 << 21
    k, t, cols = _gen(eng_mod, n, 1_000_000, 0x5c5, 1, span_ms=n // 1000)
    cfg = A.make_config(window_kind="TUMBLE", semantics="TABLE", size_ms=10_000, offset_ms=offset, aggs=C5_AGGS,
                        key_capacity=1_000_000)
    g, o = eng_mod.WindowAggregator(cfg), Oracle(cfg)
    _run_batches(g, o, k, t, cols, 4, 1000, A.agg_names(cfg), tol=lambda nm: TOL.get(nm, 0.0))
    st = g.stats()
    assert st.records_in == n and st.ingest_records == n
    g.close()
    o.close()


@pytest.mark.parametrize("rl", [False, True], ids=["dense", "record_lists"])
@pytest.mark.parametrize("kg_range", [(0, 127), (0, 63), (96, 127)], ids=["all", "p2r0", "p4r3"])
def test_c4_large_key_table_vs_oracle(eng_mod, kg_range, rl):
    """bench.py --config c4 engine shape: keys drawn from 1e8, maxParallelism 128, partial ranges get only their own
    key groups (the keyBy); dense: key capacity above 2^22 slots (single-pass primary ingest); record lists: the
    layout bench.py's 1e8-key capacity selects (FWA_CFG_RECORD_LISTS)."""
    from oracle import oracle as O
    n = 1 << 22
    k, t, cols = _gen(eng_mod, n, 100_000_000, 0xc4, 0, span_ms=n // 1000)
    lo, hi = kg_range
    if (lo, hi) != (0, 127):
        kg, _ = eng_mod.key_groups(k, 128, 1)
        sel = (kg >= lo) & (kg <= hi)
        k, t, cols = k[sel].contiguous(), t[sel].contiguous(), [c[sel].contiguous() for c in cols]
    cfg = A.make_config(window_kind="TUMBLE", size_ms=10_000, aggs=[("COUNT", 0), ("SUM_I64", 0)],
                        key_capacity=8_000_000, max_parallelism=128, kg_start=lo, kg_end=hi, record_lists=rl)
    g, o = eng_mod.WindowAggregator(cfg), O.Oracle(cfg)
    assert g.record_lists == rl
    _run_batches(g, o, k, t, cols, 3, 1000, A.agg_names(cfg))
    g.close()
    o.close()


def _full_size_conservation(eng_mod, nkeys, key_capacity):
    """The bench workload at full size: 15 x 2^26 records, async device pushes, outputs left in HBM."""
    import torch
    B, S = 1 << 26, 15
    n = B * S
    k, t, cols = _gen(eng_mod, n, nkeys, 0x5eed0001, 0, span_ms=n * 1_000_000 // 1_000_000_000)
    v = cols[0]
    bmax = t.view(S, B).max(dim=1).values.cpu().numpy()
    cfg = A.make_config(window_kind="TUMBLE", size_ms=10_000, aggs=[("COUNT", 0), ("SUM_I64", 0)],
                        key_capacity=key_capacity, output_on_device=1)
    g = eng_mod.WindowAggregator(cfg)
    cnt = torch.zeros((), dtype=torch.int64, device="cuda")
    tot = torch.zeros((), dtype=torch.int64, device="cuda")
    m = -2**63
    rows = 0
    for b in range(S):
        m = max(m, int(bmax[b]))
        wm = A.LONG_MAX if b == S - 1 else m - 1001
        g.push(k[b * B:(b + 1) * B], t[b * B:(b + 1) * B], [v[b * B:(b + 1) * B]], sync=False)
        out = g.advance_watermark_device(wm)
        rows += int(out["key"].shape[0])
        cnt += out["agg0"].sum()
        tot += out["agg1"].sum()     # int64 wrap-around, like SUM(long)
    st = g.stats()
    assert st.records_in == n
    assert int(cnt.item()) + st.late_dropped == n
    assert st.late_dropped == 0                      # bounded out-of-orderness: nothing is late
    assert int(tot.item()) == int(v.sum().item())
    assert st.rows_out == rows
    g.close()
    return rows


def test_c2_full_size_conservation(eng_mod):
    """Regression for the r01 C2 bench fault: the default bench workload end to end, checked."""
    rows = _full_size_conservation(eng_mod, 1_000_000, 1_000_000)
    assert rows > 90_000_000          # ~1M keys x ~100 windows


def test_c4_full_size_conservation(eng_mod):
    """C4 at N=1: 1e8 keys (record lists, auto-selected), 1e9 records."""
    _full_size_conservation(eng_mod, 100_000_000, 100_000_000)


@pytest.mark.parametrize("dtype", ["i64", "f32"])
def test_phase_p_paired_loads_odd_sizes_and_offsets(eng_mod, dtype):
    """Phase P reads two records per lane per column when the columns are 16-byte aligned (W16): pushes of odd
    length (the unpaired last record goes to the replay) and pushes starting at odd offsets (8-byte-aligned
    columns: the per-record load path) must both equal the oracle."""
    import torch
    from oracle.oracle import Oracle
    rng = np.random.default_rng(5)
    n = 200_001
    keys = rng.integers(0, 20_000, n).astype(np.int64)
    ts = (np.arange(n) * 5 + rng.integers(0, 3000, n)).astype(np.int64)
    vals = rng.integers(-2**40, 2**40, n).astype(np.int64) if dtype == "i64" else rng.random(n).astype(np.float32)
    aggs = [("COUNT", 0), ("SUM_I64", 0)] if dtype == "i64" else [("COUNT", 0), ("MAX_F32", 0), ("SUM_F32", 0)]
    cfg = A.make_config(window_kind="TUMBLE", size_ms=10_000, aggs=aggs, key_capacity=1 << 15)
    g, o = eng_mod.WindowAggregator(cfg), Oracle(cfg)
    names = A.agg_names(cfg)
    tk, tt, tv = (torch.from_numpy(x).cuda() for x in (keys, ts, vals))
    cuts = [0, 33_333, 33_334, 100_001, 150_000, n]              # odd / even lengths, odd / even starts
    for a_, b_ in zip(cuts[:-1], cuts[1:]):
        g.push(tk[a_:b_], tt[a_:b_], [tv[a_:b_]])
        o.push(keys[a_:b_], ts[a_:b_], [vals[a_:b_]])
        wm = int(ts[:b_].max()) - 3001 if b_ < n else A.LONG_MAX
        assert_rows_equal(g.advance_watermark(wm), o.advance_watermark(wm), names, rtol=1e-5, ctx="cut %d" % b_)
    g.close()
