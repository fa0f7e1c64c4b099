"""GPU parity of the skewed-key path: Phase P's tile pre-aggregation (PRE, partition3_kernel) against the
oracle.

A push whose key-hash partitions are skewed (a Zipf head key, or many keys in one partition: more entries than the
sub-bucket layout holds for a partition) switches the handle to PRE for the following pushes: equal (key, slice) records of a tile are
merged in LDS before bucketing, and a merged entry that still overflows is applied at once with global
atomics. Results must stay bit-exact (COUNT, BIGINT SUM) through the switch.
"""
import numpy as np
import pytest

from flink_amd import _abi as A
from helpers import assert_rows_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng_mod():
    from flink_amd import engine
    engine.lib()
    return engine


def _mix64(z):
    z = np.asarray(z, np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
    return z ^ (z >> np.uint64(31))


def _run(eng_mod, cfg, k, t, v, nb, delay, ctx, modes=None):
    from oracle.oracle import Oracle
    names = A.agg_names(cfg)
    g, o = eng_mod.WindowAggregator(cfg), Oracle(cfg)
    kh, th, vh = (x.cpu().numpy() if hasattr(x, "cpu") else x for x in (k, t, v))
    n = len(kh)
    replays = []
    for b in range(nb + 1):
        if b < nb:
            sl = slice(b * n // nb, (b + 1) * n // nb)
            assert g.push(k[sl], t[sl], [v[sl]]) == o.push(kh[sl], th[sl], [vh[sl]])
            wm = int(th[: (b + 1) * n // nb].max()) - delay - 1
        else:
            wm = A.LONG_MAX
        assert_rows_equal(g.advance_watermark(wm), o.advance_watermark(wm), names, ctx="%s wm=%d" % (ctx, wm))
        replays.append(g.stats().replay_records)
        if modes is not None and b < nb:              # the handle's pre-aggregation mode after push b
            modes.append(g.get_option("skew_merge"))
    g.close()
    o.close()
    return replays


@pytest.mark.parametrize("shape", ["hop_table", "tumble_ds"])
def test_zipf_head_key_switches_to_pre_aggregation(eng_mod, shape):
    """Zipf(1.1) over 1M keys (head key ~12 % of the records): the first push misses every slice (replayed); the
    second overflows the head key's partition's sub-buckets (those records take the v1 replay) and signals the skew;
    the following pushes pre-aggregate and replay (almost) nothing. Every watermark's rows equal the oracle's."""
    import torch
    nkeys, n = 1_000_000, 1 << 21
    w = 1.0 / np.arange(1, nkeys + 1, dtype=np.float64) ** 1.1
    cdf = np.cumsum(w) / w.sum()
    dcdf = torch.from_numpy(cdf).cuda()
    p = A.GenParams(seed_k=15, seed_t=16, seed_v=17, first_index=0, total_records=n, num_keys=nkeys, t0_ms=0,
                    span_ms=400_000, max_delay_ms=1000, key_dist=1, val_kind=0)
    p.zipf_cdf = dcdf.data_ptr()
    k = torch.empty(n, dtype=torch.int64, device="cuda")
    t = torch.empty_like(k)
    v = torch.empty_like(k)
    eng_mod.generate(p, n, k, t, v)
    torch.cuda.synchronize()
    if shape == "hop_table":
        cfg = A.make_config(window_kind="SLIDE", semantics="TABLE", size_ms=60_000, slide_ms=1_000,
                            aggs=[("COUNT", 0), ("SUM_I64", 0)], key_capacity=nkeys)
    else:
        cfg = A.make_config(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=10_000,
                            aggs=[("COUNT", 0), ("SUM_I64", 0)], key_capacity=nkeys)
    modes = []
    rep = _run(eng_mod, cfg, k, t, v, 4, 1000, shape, modes)
    # push 1 misses every slice (empty directory: all replayed) and does not see the skew; push 2 overflows on the
    # head key's partition (those records take the v1 replay) and switches the handle to pre-aggregation, which
    # pushes 3-4 then use and replay (almost) nothing
    # (the narrow Phase P, partition_nk, applies a full sub-bucket's records in place instead of replaying them)
    assert modes[0] == 0 and modes[1] == 1 and modes[3] == 1, modes
    assert rep[0] > 0 and rep[1] - rep[0] >= 0, rep
    assert rep[3] - rep[1] < (n // 4) // 100, rep


@pytest.mark.parametrize("aggs", [[("COUNT", 0), ("SUM_I64", 0)], [("COUNT", 0)]], ids=["count_sum", "count"])
def test_pre_entries_past_bucket_end_applied_with_atomics(eng_mod, aggs):
    """3000 distinct keys that all hash into ONE partition: even after the per-tile merge, a sub-bucket gets
    more entries than it holds, and the overflowing merged entries are applied with global atomics."""
    rng = np.random.default_rng(21)
    cand = rng.integers(-2**62, 2**62, 3_000_000).astype(np.int64)
    part = _mix64(cand.view(np.uint64)) >> np.uint64(64 - 9)   # capacity 2^21, SEG 4096: 512 partitions
    keys_p0 = np.unique(cand[part == 0])[:3000]
    assert len(keys_p0) == 3000
    n = 1 << 18
    k = keys_p0[rng.integers(0, len(keys_p0), n)]
    t = np.sort(rng.integers(0, 40_000, n)).astype(np.int64) - rng.integers(0, 500, n)
    v = rng.integers(-2**40, 2**40, n).astype(np.int64)
    cfg = A.make_config(window_kind="TUMBLE", semantics="TABLE", size_ms=20_000, aggs=aggs, key_capacity=1 << 20)
    _run(eng_mod, cfg, k, t, v, 4, 500, "one-partition")


def test_forced_pre_and_window_passes():
    """FWA_OPT_SKEW_MERGE / FWA_OPT_WINDOW_PASSES forced on for every handle of a child process: the pre-aggregating Phase P and the
    combiner's window passes from the first push, over Zipf keys, small HOP/CUMULATE slices and late records."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "forced_modes_check.py")], timeout=300,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
