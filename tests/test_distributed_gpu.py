"""world_size-2 keyBy pipelines with the HIP engine in every role (both ranks share the box's one
GPU; the exchange runs over gloo on host tensors since RCCL needs one GPU per rank). Raw-record and
two-phase (local pre-aggregation -> partial exchange -> global merge) plans must both reproduce one
oracle operator over the union of the sources, including late drops and MIN/MAX aggregates."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from flink_amd import _abi as A

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AGGS = [("COUNT", 0), ("SUM_I64", 0), ("MIN_I64", 0), ("MAX_I64", 0)]
CFG = dict(window_kind="SLIDE", size_ms=4000, slide_ms=1000, aggs=AGGS, key_capacity=1 << 13)
CFG_T = dict(window_kind="TUMBLE", size_ms=2000, aggs=AGGS, key_capacity=1 << 13)   # merged + fired on chip
NB, PER, DELAY = 6, 4000, 1500


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stream(seed, n):
    rng = np.random.default_rng(seed)
    keys = rng.integers(-3000, 3000, n).astype(np.int64)
    ts = np.sort(rng.integers(0, 60_000, n)).astype(np.int64) - rng.integers(0, DELAY + 1, n)
    late = rng.random(n) < 0.02
    ts[late] -= rng.integers(DELAY, 4 * DELAY, late.sum())
    vals = rng.integers(-2**40, 2**40, n).astype(np.int64)
    return keys, ts, vals


def _wms(streams):
    out = []
    for b in range(NB):
        out.append(min(int(t[: (b + 1) * PER].max()) - DELAY - 1 for _, t, _ in streams))
    return out + [A.LONG_MAX]


def _worker(rank, world, port, outdir, two_phase, routed=False, cfg=None):
    cfg = cfg or CFG
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from flink_amd.distributed import KeyedWindowPipeline, TwoPhaseKeyedWindowPipeline
    cls = TwoPhaseKeyedWindowPipeline if two_phase else KeyedWindowPipeline
    pipe = cls(rank, world, routed=True, **cfg) if routed else cls(rank, world, **cfg)
    keys, ts, vals = _stream(7 + rank, NB * PER)
    rows = []
    dev = (lambda x: torch.from_numpy(x).cuda()) if routed else torch.from_numpy  # noqa: E731
    for b in range(NB + 1):
        if b < NB:
            sl = slice(b * PER, (b + 1) * PER)
            pipe.push(dev(keys[sl]), dev(ts[sl]), [dev(vals[sl])])
            local_wm = int(ts[: (b + 1) * PER].max()) - DELAY - 1
        else:
            local_wm = A.LONG_MAX
        r = pipe.advance_watermark(local_wm)
        rows.append(np.stack([r["key"], r["win_start"], r["win_end"]] + [r["agg%d" % j] for j in range(len(AGGS))],
                             axis=1))
    dropped = pipe.engine.stats().late_dropped + (pipe.local.stats().late_dropped if two_phase else 0)
    np.save(os.path.join(outdir, "rank%d.npy" % rank), np.concatenate(rows))
    np.save(os.path.join(outdir, "drop%d.npy" % rank), np.array([dropped]))
    pipe.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("two_phase,routed,cfg", [(False, False, CFG), (True, False, CFG), (True, True, CFG),
                                                  (True, True, CFG_T)],
                         ids=["raw_records", "two_phase_partials", "two_phase_routed_device", "two_phase_routed_tumble"])
def test_two_rank_pipeline_on_gpu(tmp_path, two_phase, routed, cfg):
    """routed: the device path of the RCCL plan (fwa_drain_route -> block exchange -> fwa_fire_partials) with the
    blocks staged through the host, since both ranks share the one GPU (RCCL refuses two ranks on one device)."""
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), two_phase, routed, cfg), nprocs=world, join=True)
    got = np.concatenate([np.load(tmp_path / ("rank%d.npy" % r)) for r in range(world)])
    dropped = sum(int(np.load(tmp_path / ("drop%d.npy" % r))[0]) for r in range(world))
    from oracle.oracle import Oracle
    o = Oracle(A.make_config(**cfg))
    streams = [_stream(7 + r, NB * PER) for r in range(world)]
    exp = []
    dropped_o = 0
    for b, wm in enumerate(_wms(streams)):
        if b < NB:
            for k, t, v in streams:
                sl = slice(b * PER, (b + 1) * PER)
                dropped_o += o.push(k[sl], t[sl], [v[sl]])
        r = o.advance_watermark(wm)
        exp.append(np.stack([r["key"], r["win_start"], r["win_end"]] + [r["agg%d" % j] for j in range(len(AGGS))],
                            axis=1))
    exp = np.concatenate(exp)
    srt = lambda a: a[np.lexsort(a.T[::-1])]  # noqa: E731
    assert got.shape == exp.shape and len(exp) > 0
    assert np.array_equal(srt(got), srt(exp))
    assert dropped == dropped_o and dropped_o > 0
