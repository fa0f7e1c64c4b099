"""world_size-2 gloo test of the key-group-partitioned pipeline (flink_amd.distributed): the keyBy
all-to-all + MIN-watermark protocol must give exactly the single-operator result. The per-rank
engine is the oracle here (no GPU in this container); on the GPU box it is the HIP engine."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from flink_amd import _abi as A

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stream(seed, n):
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, 5000, n).astype(np.int64)
    ts = np.sort(rng.integers(0, 100_000, n)).astype(np.int64) - rng.integers(0, 2000, n)
    vals = rng.integers(-1000, 1000, n).astype(np.int64)
    return keys, ts, vals


class _LocalPreAgg:
    """Test-side CPU stand-in for the GPU pre-aggregator role (fwa_drain_partials semantics, tumbling
    COUNT + SUM_I64): drops records whose window fired at the current watermark, buffers the rest,
    drain(wm) emits one (key, slice_start, count, sum) partial per key and complete slice."""

    def __init__(self, cfg):
        self.size = cfg.size_ms
        self.wm = A.LONG_MIN
        self.buf = []

    def push(self, keys, ts, cols=()):
        start = ts - np.mod(ts, self.size)
        ok = start + self.size - 1 > self.wm
        self.buf.append((keys[ok], start[ok], cols[0][ok]))
        return int((~ok).sum())

    def drain_partials(self, wm):
        self.wm = max(self.wm, wm)
        if not self.buf:
            k = s = v = np.zeros(0, np.int64)
        else:
            k, s, v = (np.concatenate(c) for c in zip(*self.buf))
        done = s + self.size - 1 <= self.wm
        self.buf = [(k[~done], s[~done], v[~done])]
        groups = {}
        for key, st, val in zip(k[done].tolist(), s[done].tolist(), v[done].tolist()):
            c, t = groups.get((key, st), (0, 0))
            groups[(key, st)] = (c + 1, t + val)
        items = sorted(groups.items())
        arr = lambda f: np.array([f(it) for it in items], dtype=np.int64)  # noqa: E731
        return {"key": arr(lambda it: it[0][0]), "slice_start": arr(lambda it: it[0][1]),
                "count": arr(lambda it: it[1][0]), "acc0": arr(lambda it: it[1][0]), "acc1": arr(lambda it: it[1][1])}

    def close(self):
        pass


class _OracleFromPartials:
    """Test-side global role: merges partials into the oracle by re-expanding each (count c, sum s)
    partial into c records at slice_start (one carrying s, the rest 0) -- exact for COUNT + SUM."""

    def __init__(self, cfg):
        from oracle.oracle import Oracle
        self.o = Oracle(cfg)

    def push_partials(self, keys, slice_ts, count, accs, hidden=()):
        rep = np.repeat(np.arange(len(keys)), count)
        first = np.r_[True, rep[1:] != rep[:-1]] if len(rep) else np.zeros(0, bool)
        vals = np.where(first, np.asarray(accs[1])[rep], 0).astype(np.int64)
        return self.o.push(np.asarray(keys)[rep], np.asarray(slice_ts)[rep], [vals])

    def advance_watermark(self, wm):
        return self.o.advance_watermark(wm)

    def close(self):
        self.o.close()


def _worker(rank, world, port, outdir, two_phase=False, pipelined=False):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from flink_amd.distributed import KeyedWindowPipeline
    from oracle import oracle as O
    L = O.lib()

    def router(keys):  # KeyGroupStreamPartitioner.selectChannel restated through the oracle
        return torch.tensor([L.or_operator_index(128, world, L.or_key_group(int(k), 0, 0, 128)) for k in keys.tolist()],
                            dtype=torch.int64)

    kw = dict(router=router, window_kind="TUMBLE", size_ms=5000, aggs=[("COUNT", 0), ("SUM_I64", 0)])
    if two_phase:
        from flink_amd.distributed import TwoPhaseKeyedWindowPipeline
        pipe = TwoPhaseKeyedWindowPipeline(rank, world, engine_factory=_OracleFromPartials,
                                           local_factory=_LocalPreAgg, **kw)
    else:
        pipe = KeyedWindowPipeline(rank, world, engine_factory=O.Oracle, **kw)
    keys, ts, vals = _stream(42 + rank, 6000)   # each rank is one source subtask
    rows = []
    nb = 4
    batch = lambda b: (torch.from_numpy(keys[b * 1500:(b + 1) * 1500]), torch.from_numpy(ts[b * 1500:(b + 1) * 1500]),  # noqa: E731
                       [torch.from_numpy(vals[b * 1500:(b + 1) * 1500])])
    if pipelined:
        pipe.push(*batch(0))
    for b in range(nb + 1):
        if b < nb:
            if not pipelined:
                pipe.push(*batch(b))
            local_wm = int(ts[: (b + 1) * 1500].max()) - 2001
        else:
            local_wm = A.LONG_MAX
        if pipelined:       # the next batch enters the local pre-aggregator during this watermark's exchange
            r = pipe.advance_watermark(local_wm, then_push=batch(b + 1) if b + 1 < nb else None)
        else:
            r = pipe.advance_watermark(local_wm)
        rows.append(np.stack([r["key"], r["win_start"], r["win_end"], r["agg0"], r["agg1"]], axis=1))
    np.save(os.path.join(outdir, "rank%d.npy" % rank), np.concatenate(rows))
    pipe.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("two_phase,pipelined", [(False, False), (True, False), (True, True)],
                         ids=["raw_records", "two_phase_partials", "two_phase_pipelined"])
def test_two_rank_keyby_pipeline_matches_single_operator(tmp_path, two_phase, pipelined):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), two_phase, pipelined), nprocs=world, join=True)
    got = np.concatenate([np.load(tmp_path / ("rank%d.npy" % r)) for r in range(world)])
    # reference: one operator over the union of both sources, watermark = min over sources per step
    from oracle.oracle import Oracle
    cfg = A.make_config(window_kind="TUMBLE", size_ms=5000, aggs=[("COUNT", 0), ("SUM_I64", 0)])
    o = Oracle(cfg)
    streams = [_stream(42 + r, 6000) for r in range(world)]
    exp = []
    for b in range(5):
        if b < 4:
            for k, t, v in streams:
                sl = slice(b * 1500, (b + 1) * 1500)
                o.push(k[sl], t[sl], [v[sl]])
            wm = min(int(t[: (b + 1) * 1500].max()) - 2001 for k, t, v in streams)
        else:
            wm = A.LONG_MAX
        r = o.advance_watermark(wm)
        exp.append(np.stack([r["key"], r["win_start"], r["win_end"], r["agg0"], r["agg1"]], axis=1))
    exp = np.concatenate(exp)
    key = lambda a: a[np.lexsort(a.T[::-1])]
    assert got.shape == exp.shape
    assert np.array_equal(key(got), key(exp))
    # every key's rows live on exactly the rank owning its key group
    ranks = [np.load(tmp_path / ("rank%d.npy" % r)) for r in range(world)]
    assert not (set(ranks[0][:, 0].tolist()) & set(ranks[1][:, 0].tolist()))


def test_choose_exchange_plan():
    """Two-phase partials unless the key space puts the engine in its record-list regime (C4), where a step's partial
    rows would outnumber and outweigh its records."""
    from flink_amd.distributed import choose_exchange
    assert choose_exchange(dict(key_capacity=1_000_000)) == "partials"
    assert choose_exchange(dict(key_capacity=100_000_000)) == "raw"
    assert choose_exchange(dict(key_capacity=4096, record_lists=True)) == "raw"


def _valve_worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import flink_amd.distributed as D
    from oracle import oracle as O
    created = []
    real_new_group = dist.new_group

    def counting_new_group(*a, **kw):
        created.append(kw.get("ranks"))
        return real_new_group(*a, **kw)
    D.dist.get_backend = lambda group=None: "nccl"      # take the RCCL branch; the group itself stays gloo
    D.dist.new_group = counting_new_group
    kw = dict(router=lambda k: torch.zeros(len(k), dtype=torch.int64), window_kind="TUMBLE", size_ms=5000,
              aggs=[("COUNT", 0)])
    p1 = D.KeyedWindowPipeline(rank, world, engine_factory=O.Oracle, **kw)
    p2 = D.KeyedWindowPipeline(rank, world, engine_factory=O.Oracle, **kw)
    assert p1.wm_group is p2.wm_group and created == [[0, 1]], created
    assert p1.global_watermark(100 + rank) == 100 and p2.global_watermark(7 - rank) == 6
    p1.close()
    p2.close()
    dist.destroy_process_group()


def test_valve_group_created_once_per_rank_set():
    """under RCCL the watermark valve's gloo group is created once per rank set and shared by every
    pipeline built on it (no group per pipeline instance piling up; two pipelines on one group do not hang)."""
    mp.spawn(_valve_worker, args=(2, _free_port()), nprocs=2, join=True)


def test_owner_key_capacity_share():
    """distributed.owner_key_capacity: an owner's key table sized to its key groups' share (+25 % and a slack), never
    above the job's capacity; record-list sized key spaces keep theirs (the capacity selects that layout)."""
    from flink_amd.distributed import owner_key_capacity
    assert owner_key_capacity(1_000_000, 16, 128) == int(125_000 * 1.25) + 4096
    assert owner_key_capacity(8192, 64, 128) == 8192                 # share + slack above the job's capacity
    assert owner_key_capacity(1 << 25, 16, 128) == 1 << 25           # record lists
    assert owner_key_capacity(1_000_000, 128, 128) == 1_000_000      # one owner of every key group
    assert owner_key_capacity(0, 16, 128) == 0                       # engine default
    # the share covers the owner's keys: key groups spread keys evenly (murmur), 8 owners of 200K random keys
    from flink_amd.keygroups import key_group_range_for_operator
    from oracle.oracle import lib as olib
    L = olib()
    keys = np.random.default_rng(3).integers(-2**62, 2**62, 200_000)
    kg = np.array([L.or_key_group(int(k), 0, 0, 128) for k in keys.tolist()])
    for r in range(8):
        lo, hi = key_group_range_for_operator(128, 8, r)
        assert int(((kg >= lo) & (kg <= hi)).sum()) <= owner_key_capacity(200_000, hi - lo + 1, 128)
