"""GPU tests: checkpoint / restore / rescale of DataStream state keyed by String keys (FWA_KEY_PREHASHED).

Reference behaviour: WindowOperator is generic in its key type (WindowOperator.java:179-208) and the heap backend
checkpoints any key per key group, the group being assignToKeyGroup(key.hashCode(), maxParallelism)
(HeapSnapshotStrategy.java:154-179, KeyGroupRangeAssignment.java:63-76); a restored or rescaled job emits exactly the
windows of an uninterrupted run (EventTimeWindowCheckpointingITCase.java:759-810). The engine receives such keys as
64-bit ids with the caller's key.hashCode() beside them; it keeps each key's hash (by kid) so fwa_snapshot can place
the state in key groups and carries the hash in the blob, so a restore into other key-group ranges places it again.
Here the keys are Java Strings ("user-<i>"), ids their dictionary positions, hashes String.hashCode(); every test runs
1 subtask -> 2 (scale-out) -> 1 (scale-in) against one uninterrupted oracle operator over the whole stream.
"""
import numpy as np
import pytest

from flink_amd import _abi as A
from flink_amd import snapshot as S
from helpers import assert_rows_equal, java_hash_code
from test_gpu_parity import CONFIGS, I64_AGGS
from test_snapshot_gpu import batches

pytestmark = pytest.mark.gpu

NAMES = ["user-%d" % i for i in range(900)] + ["", "é", "ümlaut-key", "a" * 40]
HASH = np.array([java_hash_code(s, "String") for s in NAMES], np.int32)


@pytest.fixture(scope="module")
def eng_mod():
    from flink_amd import engine
    engine.lib()
    return engine


def _stream(seed, n=24_000):
    """String-keyed stream: ids into NAMES (two ids hash alike when their strings do), ts, value columns."""
    rng = np.random.default_rng(seed)
    ids = rng.integers(0, len(NAMES), n).astype(np.int64)
    base = np.sort(rng.integers(0, 40_000, n)).astype(np.int64)
    ts = base - rng.integers(0, 1001, n)
    late = rng.random(n) < 0.02
    ts[late] -= rng.integers(1000, 4001, late.sum())
    vi = rng.integers(-2**40, 2**40, n).astype(np.int64)
    vf = rng.random(n).astype(np.float32) * 100
    vd = rng.random(n) * 1000.0 - 500.0
    return ids, ts, vi, vf, vd


def _run(eng_mod, base, seed):
    from flink_amd import keygroups as KG
    from oracle.oracle import Oracle
    names = A.agg_names(A.make_config(**base))
    ranges = [KG.key_group_range_for_operator(128, 2, i) for i in range(2)]
    cfg1 = A.make_config(**base)
    cfgs2 = [A.make_config(kg_start=r[0], kg_end=r[1], **base) for r in ranges]
    o = Oracle(cfg1)
    bs = batches(_stream(seed), 9, 1000)

    def route(k):
        _, op = eng_mod.key_groups(k, 128, 2, key_kind=A.KEY_PREHASHED, key_hash=HASH[k])
        return [op == i for i in range(2)]

    def fire(handles, wm):
        parts = [h.advance_watermark(wm) for h in handles]
        return {f: np.concatenate([p[f] for p in parts]) for f in parts[0]}

    def step(handles, b, k, t, cols, wm, split):
        o.push(k, t, cols, key_hash=HASH[k])
        masks = route(k) if split else [np.ones(len(k), bool)]
        for h, m in zip(handles, masks):
            h.push(k[m], t[m], [c[m] for c in cols], key_hash=HASH[k[m]])
        assert_rows_equal(fire(handles, wm), o.advance_watermark(wm), names, ctx="b=%d" % b)

    one = eng_mod.WindowAggregator(cfg1)
    for b, (k, t, cols, wm) in enumerate(bs[:3]):
        step([one], b, k, t, cols, wm, False)
    blob = one.snapshot()
    snap = S.parse(blob)
    assert snap["n"] > 0 and len(snap["key_hash"]) == snap["n"]
    assert np.array_equal(snap["key_hash"], HASH[snap["key"]])      # the hash each key was pushed with
    one.close()
    two = [eng_mod.WindowAggregator(c) for c in cfgs2]               # scale-out: 1 -> 2
    for h in two:
        h.restore(blob)
    for b, (k, t, cols, wm) in enumerate(bs[3:6], start=3):
        step(two, b, k, t, cols, wm, True)
    blobs = [h.snapshot() for h in two]
    for h in two:
        h.close()
    one = eng_mod.WindowAggregator(cfg1)                             # scale-in: 2 -> 1
    one.restore(blobs)
    for b, (k, t, cols, wm) in enumerate(bs[6:], start=6):
        step([one], b, k, t, cols, wm, False)
    one.close()


@pytest.mark.parametrize("ci", [0, 3, 7, 8, 9])
def test_string_keyed_snapshot_rescale_restore(eng_mod, ci):
    """TUMBLE, SLIDE and SESSION (with allowed lateness) DataStream windows over String keys."""
    _run(eng_mod, dict(aggs=I64_AGGS, key_capacity=4096, key_kind=A.KEY_PREHASHED, **CONFIGS[ci]), 900 + ci)


def test_string_keyed_reduce_snapshot_rescale_restore(eng_mod):
    """WindowedStream.sum(1) over String keys: the restore pushes each key's reduced element back with its hash."""
    _run(eng_mod, dict(aggs=[("SUM_I64", 0), ("FIRST_32", 1), ("FIRST_64", 2)], reduce=True, key_capacity=4096,
                       key_kind=A.KEY_PREHASHED, **CONFIGS[0]), 990)


def test_prehashed_record_lists_snapshot_refused(eng_mod):
    """Record lists keep no key table, hence no per-key hash: their PREHASHED snapshot is refused, not wrong."""
    g = eng_mod.WindowAggregator(A.make_config(aggs=I64_AGGS, key_kind=A.KEY_PREHASHED, record_lists=True,
                                               key_capacity=4096, **CONFIGS[0]))
    k = np.arange(10, dtype=np.int64)
    g.push(k, k * 10, [k, k.astype(np.float32), k.astype(np.float64)], key_hash=HASH[k])
    with pytest.raises(eng_mod.EngineError):
        g.snapshot()
    g.close()
