"""2-rank rehearsal of the two-phase pipeline's device path on ONE GPU (both ranks on cuda:0; RCCL refuses two ranks
on one device, so the group is gloo and the row blocks are staged through the host): the routed drain
(fwa_drain_route), the count exchange, the block all-to-all and the owner's fwa_fire_partials with the next batch
pipelined, checked against one oracle operator over the union of both ranks' streams."""
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from flink_amd import _abi as A  # noqa: E402

CFG = dict(window_kind="TUMBLE", size_ms=2000, aggs=[("COUNT", 0), ("SUM_I64", 0), ("MAX_I64", 0)], key_capacity=1 << 14)
NB, PER = 6, 20000


def stream(seed):
    rng = np.random.default_rng(seed)
    n = NB * PER
    keys = rng.integers(-5000, 5000, n).astype(np.int64)
    ts = np.sort(rng.integers(0, 60_000, n)).astype(np.int64) - rng.integers(0, 500, n)
    vals = rng.integers(-2**40, 2**40, n).astype(np.int64)
    return keys, ts, vals


def worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from flink_amd.distributed import TwoPhaseKeyedWindowPipeline
    pipe = TwoPhaseKeyedWindowPipeline(rank, world, routed=True, **CFG)
    assert pipe.routed_drain
    keys, ts, vals = stream(11 + rank)
    rows = []
    batch = lambda b: (torch.from_numpy(keys[b * PER:(b + 1) * PER]).cuda(),  # noqa: E731
                       torch.from_numpy(ts[b * PER:(b + 1) * PER]).cuda(), [torch.from_numpy(vals[b * PER:(b + 1) * PER]).cuda()])
    pipe.push(*batch(0))
    for b in range(NB + 1):
        wm = int(ts[: (b + 1) * PER].max()) - 501 if b < NB else A.LONG_MAX
        # pipelined as bench.py does: batch b+1 enters the local engine during this watermark's exchange
        r = pipe.advance_watermark(wm, then_push=batch(b + 1) if b + 1 < NB else None)
        rows.append(np.stack([r["key"], r["win_start"], r["agg0"], r["agg1"], r["agg2"]], axis=1))
    np.save(os.path.join(out, "r%d.npy" % rank), np.concatenate(rows))
    print("rank %d fire_partials on chip: %d" % (rank, pipe.engine.get_option("fire_partials")), flush=True)
    pipe.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    import tempfile
    out = tempfile.mkdtemp()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(worker, args=(2, port, out), nprocs=2, join=True)
    got = np.concatenate([np.load(os.path.join(out, "r%d.npy" % r)) for r in range(2)])
    from oracle.oracle import Oracle
    o = Oracle(A.make_config(**CFG))
    st = [stream(11 + r) for r in range(2)]
    exp = []
    for b in range(NB + 1):
        if b < NB:
            for k, t, v in st:
                sl = slice(b * PER, (b + 1) * PER)
                o.push(k[sl], t[sl], [v[sl]])
            wm = min(int(t[: (b + 1) * PER].max()) - 501 for _, t, _ in st)
        else:
            wm = A.LONG_MAX
        r = o.advance_watermark(wm)
        exp.append(np.stack([r["key"], r["win_start"], r["agg0"], r["agg1"], r["agg2"]], axis=1))
    exp = np.concatenate(exp)
    srt = lambda a: a[np.lexsort(a.T[::-1])]  # noqa: E731
    ok = got.shape == exp.shape and np.array_equal(srt(got), srt(exp))
    print("2-rank two-phase pipeline on ONE GPU over gloo (host-staged row blocks, not RCCL; routed drain, fire_partials) "
          "rows %d vs oracle %d: %s" % (len(got), len(exp), "EQUAL" if ok else "DIFFERENT"))
    sys.exit(0 if ok else 1)
