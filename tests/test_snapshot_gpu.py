"""GPU tests: checkpoint / restore of the window state (fwa_snapshot / fwa_restore).

Reference behaviour: the keyed window state is snapshotted per key group (HeapSnapshotStrategy.java:154-179)
and the SlicingWindowOperator watermark as union list state whose MIN is taken on restore
(SlicingWindowOperator.java:186-209). The end-to-end invariant follows
EventTimeWindowCheckpointingITCase.java:759-810: a job restored from a checkpoint emits exactly the
windows of an uninterrupted run. Each test checks the rows against the oracle (one uninterrupted
operator over the whole stream), including rescaling 2 -> 1 and 1 -> 2 subtasks.
"""
import numpy as np
import pytest

from flink_amd import _abi as A
from flink_amd import snapshot as S
from helpers import assert_rows_equal
from test_gpu_parity import CONFIGS, I64_AGGS, F64_AGGS, random_stream, tol

pytestmark = pytest.mark.gpu

SLICING = [i for i, c in enumerate(CONFIGS) if c["window_kind"] != "SESSION"]
SESSIONS = [i for i, c in enumerate(CONFIGS) if c["window_kind"] == "SESSION"]


def batches(stream, nb, delay):
    keys, ts, vi, vf, vd = stream
    n = len(keys)
    max_ts = -2**63
    out = []
    for b in range(nb):
        sl = slice(b * n // nb, (b + 1) * n // nb)
        max_ts = max(max_ts, int(ts[sl].max()))
        wm = max_ts - delay - 1 if b < nb - 1 else A.LONG_MAX
        out.append((keys[sl], ts[sl], [vi[sl], vf[sl], vd[sl]], wm))
    return out


@pytest.fixture(scope="module")
def eng_mod():
    from flink_amd import engine
    engine.lib()
    return engine


@pytest.mark.parametrize("ci", SLICING + SESSIONS)
@pytest.mark.parametrize("aggs", [I64_AGGS, F64_AGGS], ids=["i64", "f64"])
def test_snapshot_restore_resumes_exactly(eng_mod, ci, aggs):
    """Snapshot after batch 4 of 8, restore into a fresh handle, continue: rows equal the oracle's."""
    from oracle.oracle import Oracle
    cfg = A.make_config(aggs=aggs, key_capacity=4096, **CONFIGS[ci])
    names = A.agg_names(cfg)
    g, o = eng_mod.WindowAggregator(cfg), Oracle(cfg)
    dg = do = 0
    for b, (k, t, cols, wm) in enumerate(batches(random_stream(500 + ci, 24_000, 400, 40_000, 1000), 8, 1000)):
        dg += g.push(k, t, cols)
        do += o.push(k, t, cols)
        if b == 4:   # checkpoint barrier between the push and the watermark
            blob = g.snapshot()
            snap = S.parse(blob)
            assert snap["n"] > 0 and snap["watermark"] == g.stats().current_watermark
            assert snap["kg_offsets"][-1] == snap["n"]
            # rows the old subtask already produced before the barrier (late firings inside processElement)
            pre = g.advance_watermark(g.stats().current_watermark)
            g.close()
            g = eng_mod.WindowAggregator(cfg)
            g.restore(blob)
            post = g.advance_watermark(wm)
            got = {f: np.concatenate([pre[f], post[f]]) for f in post}
            assert_rows_equal(got, o.advance_watermark(wm), names, rtol=tol, ctx="b=%d" % b)
            continue
        assert_rows_equal(g.advance_watermark(wm), o.advance_watermark(wm), names, rtol=tol, ctx="b=%d" % b)
    assert dg == do


@pytest.mark.parametrize("ci", [0, 3, 5, 6] + [i for i in SESSIONS if not CONFIGS[i].get("allowed_lateness_ms")])
def test_snapshot_rescale_2_to_1_and_1_to_2(eng_mod, ci):
    """Two subtasks (key groups [0,63], [64,127]) snapshot; restore both into one subtask (scale-in)
    and one subtask's snapshot into two (scale-out). The union of emitted rows equals the oracle."""
    from flink_amd import keygroups as KG
    from oracle.oracle import Oracle
    base = dict(aggs=I64_AGGS, key_capacity=4096, **CONFIGS[ci])
    names = A.agg_names(A.make_config(**base))
    ranges = [KG.key_group_range_for_operator(128, 2, i) for i in range(2)]
    cfgs2 = [A.make_config(kg_start=r[0], kg_end=r[1], **base) for r in ranges]
    cfg1 = A.make_config(**base)
    o = Oracle(cfg1)
    sub = [eng_mod.WindowAggregator(c) for c in cfgs2]
    bs = batches(random_stream(700 + ci, 24_000, 400, 40_000, 1000), 8, 1000)

    def route(k):
        _, op = eng_mod.key_groups(k, 128, 2)
        return [op == i for i in range(2)]

    def fire(handles, wm):
        parts = [h.advance_watermark(wm) for h in handles]
        return {f: np.concatenate([p[f] for p in parts]) for f in parts[0]}

    for b, (k, t, cols, wm) in enumerate(bs[:4]):
        o.push(k, t, cols)
        for h, m in zip(sub, route(k)):
            h.push(k[m], t[m], [c[m] for c in cols])
        assert_rows_equal(fire(sub, wm), o.advance_watermark(wm), names, rtol=tol, ctx="b=%d" % b)
    blobs = [h.snapshot() for h in sub]
    for h in sub:
        h.close()
    one = eng_mod.WindowAggregator(cfg1)           # scale-in: 2 -> 1
    one.restore(blobs)
    for b, (k, t, cols, wm) in enumerate(bs[4:6], start=4):
        o.push(k, t, cols)
        one.push(k, t, cols)
        assert_rows_equal(fire([one], wm), o.advance_watermark(wm), names, rtol=tol, ctx="b=%d" % b)
    blob1 = one.snapshot()
    one.close()
    two = [eng_mod.WindowAggregator(c) for c in cfgs2]   # scale-out: 1 -> 2
    for h in two:
        h.restore(blob1)
    for b, (k, t, cols, wm) in enumerate(bs[6:], start=6):
        o.push(k, t, cols)
        for h, m in zip(two, route(k)):
            h.push(k[m], t[m], [c[m] for c in cols])
        assert_rows_equal(fire(two, wm), o.advance_watermark(wm), names, rtol=tol, ctx="b=%d" % b)


def test_restore_rejects_mismatch_and_used_handle(eng_mod):
    cfg = A.make_config(aggs=I64_AGGS, key_capacity=1024, **CONFIGS[0])
    g = eng_mod.WindowAggregator(cfg)
    k = np.arange(100, dtype=np.int64)
    g.push(k, k * 10, [k, k.astype(np.float32), k.astype(np.float64)])
    blob = g.snapshot()
    with pytest.raises(eng_mod.EngineError):
        g.restore(blob)                             # handle already has state
    other = eng_mod.WindowAggregator(A.make_config(aggs=I64_AGGS, key_capacity=1024, **CONFIGS[3]))
    with pytest.raises(eng_mod.EngineError):
        other.restore(blob)                         # different window configuration
    bad = bytearray(blob)
    bad[0] ^= 1
    fresh = eng_mod.WindowAggregator(cfg)
    with pytest.raises(eng_mod.EngineError):
        fresh.restore(bytes(bad))
    fresh.restore(blob)
    assert fresh.stats().current_watermark == g.stats().current_watermark
