"""Benchmark: records/sec aggregated by the MI355X window engine (BASELINE.json metric).

Workload (N=1): config C2 of BASELINE.json -- event-time tumbling 10 s window, COUNT + SUM(long), over
synthetic (long key, long ts, long val) records, 1M uniform keys, batches of 2^26 records (defaults as the driver
runs it: 5 warm-up + 20 timed = 1.34e9 timed records), bounded out-of-orderness D = 1 s,
wm = max_ts - D - 1 after every batch, final wm = Long.MAX.
A step = one batch pushed through the engine + the watermark advance that fires its windows. Inputs are
generated into HBM before timing; outputs stay in HBM.

N>1 (torchrun, one rank per GPU): weak scaling -- every rank sources a stream of the same size and
event-time range (its own key/value seeds), records are routed to their key-group owner with RCCL
all_to_all (flink_amd.distributed, the keyBy shuffle), watermark = MIN-allreduce over ranks.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
C2_RECORDS = 1_000_000_000
C2_SPAN_MS = 1_000_000   # 1000 s of event time for 1e9 records


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)     # the driver's --steps 20 --warmup 5
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1 << 26)
    ap.add_argument("--keys", type=int, default=1_000_000)
    ap.add_argument("--window-ms", type=int, default=10_000)
    ap.add_argument("--delay-ms", type=int, default=1000)
    ap.add_argument("--cpu-sample", type=int, default=6 << 26)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive (host pinned input) leg")
    ap.add_argument("--pcie-batches", type=int, default=3)
    ap.add_argument("--no-wire", action="store_true", help="skip the wire-input (network bytes in HBM) leg")
    ap.add_argument("--wire-batches", type=int, default=4)
    ap.add_argument("--no-wide", action="store_true", help="skip the 64-bit-key leg (C2 without narrow entries)")
    ap.add_argument("--wide-batches", type=int, default=8)
    ap.add_argument("--config", choices=["c2", "c3", "c4", "c5", "c5s", "reduce"], default="c2",
                    help="c2: tumbling 10s COUNT+SUM(long), 1M uniform keys (the metric's workload); "
                         "c3: HOP 60s/1s (Table slicing), Zipf(1.1) keys over 1M items; "
                         "c4: tumbling 10s COUNT+SUM(long), 100M uniform keys, maxParallelism 128; "
                         "c5: Table TUMBLE 10s TVF COUNT, SUM(double), AVG(double), MAX(float), MAX(double); "
                         "c5s: DataStream session windows (gap 5s), same float aggregates; "
                         "reduce: the C2 stream through a DataStream built-in reduction, WindowedStream.sum(1) over "
                         "Tuple3<Long key, Long val, Long ts> (the reduced tuple keeps the first element's ts)")
    ap.add_argument("--sync-fire", action="store_true",
                    help="N=1: wait for each watermark's rows before the next batch is handed over "
                         "(fwa_advance_watermark); default: fwa_advance_watermark_async, the rows taken after the next "
                         "batch was handed over, so the next push's host work overlaps the fire (warm-up the same way)")
    ap.add_argument("--reduce-op", choices=["sum", "max_by"], default="sum",
                    help="--config reduce: WindowedStream.sum(1) (default) or maxBy(1) (the by-value selection passes)")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="fwa_set_option on the measured engine(s) (flink_amd.engine.OPTIONS), e.g. profile=1")
    ap.add_argument("--exchange", choices=["auto", "partials", "raw"], default="auto",
                    help="N>1 keyBy plan: two-phase partial accumulators or raw records; auto: the plan "
                         "flink_amd.distributed.choose_exchange picks for the configuration (raw for C4's 1e8 keys)")
    args = ap.parse_args()
    if args.config == "c4" and args.keys == 1_000_000:
        args.keys = 100_000_000
    fp = args.config in ("c5", "c5s")   # float value columns (f32 + f64)

    from flink_amd import _abi as A
    from flink_amd import engine as E
    for o in args.option:                           # A/B and diagnostic options, every handle of this run
        k, v = o.split("=", 1)
        E.DEFAULT_OPTIONS[k] = int(v)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # FWA_DIST_BACKEND=gloo: rehearsal of the N>1 path with several ranks sharing one GPU (the exchange then
    # runs over gloo on host tensors); the driver's multi-GPU runs use RCCL ("nccl"), one GPU per rank
    backend = os.environ.get("FWA_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local_rank = local_rank % max(1, torch.cuda.device_count())
    if world != args.gpus:
        log("note: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    B = args.batch
    S = args.warmup + args.steps
    n_rank = S * B
    # event-time density of C2 (1e6 records per second of event time) on every rank
    span = n_rank * C2_SPAN_MS // C2_RECORDS
    p = A.GenParams(seed_k=0x5eed0001 ^ (rank * 0x9E3779B97F4A7C15 & 0xFFFFFFFFFFFFFFFF),
                    seed_t=0x5eed0002 + rank, seed_v=0x5eed0003 + rank, first_index=0, total_records=n_rank,
                    num_keys=args.keys, t0_ms=1_700_000_000_000, span_ms=span, max_delay_ms=args.delay_ms,
                    key_dist=1 if args.config == "c3" else 0, val_kind=1 if fp else 0)
    if args.config == "c3":   # Zipf(1.1) CDF over the key ids, sampled bit-identically by the device generator
        w = 1.0 / np.arange(1, args.keys + 1, dtype=np.float64) ** 1.1
        zcdf = torch.from_numpy(np.cumsum(w) / w.sum()).to(dev)
        p.zipf_cdf = zcdf.data_ptr()
    log("rank %d/%d generating %d records (%.1f GB) in HBM" % (rank, world, n_rank, n_rank * 24 / 1e9))
    keys = torch.empty(n_rank, dtype=torch.int64, device=dev)
    ts = torch.empty_like(keys)
    if fp:
        vals = torch.empty(n_rank, dtype=torch.float32, device=dev)
        vals_d = torch.empty(n_rank, dtype=torch.float64, device=dev)
        E.generate(p, n_rank, keys, ts, None, vals, vals_d, device=local_rank)
    else:
        vals = torch.empty_like(keys)
        E.generate(p, n_rank, keys, ts, vals, device=local_rank)
    torch.cuda.synchronize()
    bmax = ts.view(S, B).max(dim=1).values.cpu().numpy()
    wms = []
    m = -2**63
    for b in range(S):
        m = max(m, int(bmax[b]))
        wms.append(m - args.delay_ms - 1)          # BoundedOutOfOrdernessWatermarks.onPeriodicEmit
    wms[-1] = A.LONG_MAX                           # final watermark flushes every window

    win_kw = dict(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=args.window_ms)
    if args.config == "c3":
        win_kw = dict(window_kind="SLIDE", semantics="TABLE", size_ms=60_000, slide_ms=1_000)
    aggs = [("COUNT", 0), ("SUM_I64", 0)]
    if args.config == "reduce":   # FWA_CFG_REDUCE: field 1 summed, field 2 the window's first element's
        aggs = [("SUM_I64", 0), ("FIRST_64", 1)]
        if args.reduce_op == "max_by":   # maxBy(1): the element with the largest f1 (ties: the first), f2 its own
            aggs = [("MAXBY_I64", 0), ("SEL_64", 1)]
    if fp:   # C5: column 0 = f (FLOAT), column 1 = d (DOUBLE)
        aggs = [("COUNT", 0), ("SUM_F64", 1), ("AVG_F64", 1), ("MAX_F32", 0), ("MAX_F64", 1)]
        win_kw = dict(window_kind="TUMBLE", semantics="TABLE", size_ms=args.window_ms)
        if args.config == "c5s":
            win_kw = dict(window_kind="SESSION", semantics="DATASTREAM", gap_ms=5_000)
    cfg_kw = dict(**win_kw,
                  aggs=aggs, key_capacity=int(args.keys * float(os.environ.get("FWA_KCAP", "1"))),
                  output_on_device=1, device=local_rank, reduce=args.config == "reduce")
    cols_of = (lambda b: [vals[b * B:(b + 1) * B], vals_d[b * B:(b + 1) * B]]) if fp else \
        (lambda b: [vals[b * B:(b + 1) * B], ts[b * B:(b + 1) * B]]) if args.config == "reduce" else \
        (lambda b: [vals[b * B:(b + 1) * B]])
    pipelined = None
    if args.exchange == "auto":
        from flink_amd.distributed import choose_exchange
        args.exchange = "raw" if args.config == "reduce" else choose_exchange(cfg_kw)   # reductions: no partials
    if world > 1:
        from flink_amd.distributed import KeyedWindowPipeline, TwoPhaseKeyedWindowPipeline
        cls = TwoPhaseKeyedWindowPipeline if args.exchange == "partials" else KeyedWindowPipeline
        pipe = cls(rank, world, **cfg_kw)
        eng = pipe.local if args.exchange == "partials" else pipe.engine   # the ingest path being measured
        engines = [pipe.engine] + ([pipe.local] if args.exchange == "partials" else [])
        batch_of = lambda b: (keys[b * B:(b + 1) * B], ts[b * B:(b + 1) * B], cols_of(b))  # noqa: E731
        push = lambda b: pipe.push(*batch_of(b))  # noqa: E731
        fire = lambda b: pipe.advance_watermark(wms[b], device_output=True)["key"].shape[0]  # noqa: E731
        if args.exchange == "partials":
            # software pipelining across steps: batch b+1 enters the local pre-aggregator while batch b's partials
            # are exchanged, merged and fired (same per-engine call order; every timed batch is pushed and fired
            # inside the timed region)
            pipelined = lambda b, nxt: pipe.advance_watermark(  # noqa: E731
                wms[b], device_output=True, then_push=batch_of(nxt) if nxt is not None else None)["key"].shape[0]
    else:
        eng = E.WindowAggregator(A.make_config(**cfg_kw))
        views = [(keys[b * B:(b + 1) * B], ts[b * B:(b + 1) * B], cols_of(b)) for b in range(S)]
        push = lambda b: eng.push(*views[b], sync=False)  # noqa: E731
        # fired rows stay in HBM (engine-owned device columns); only the row count comes back
        fire = lambda b: eng.advance_watermark_raw(wms[b]).n_rows  # noqa: E731
        engines = [eng]

    rows = 0
    async_fire = world == 1 and not args.sync_fire
    for b in range(args.warmup):
        push(b)
        if async_fire:        # the same calls as the timed loop (output buffers grown, modes settled before timing)
            if b > 0:
                rows += eng.fired_output_raw().n_rows
            eng.advance_watermark_async(wms[b])
        else:
            rows += fire(b)
    if async_fire and args.warmup > 0:
        rows += eng.fired_output_raw().n_rows
    for x in engines:
        x.reset_timers()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rows_t = 0
    dropped = 0
    if pipelined is not None:
        push(args.warmup)
        for b in range(args.warmup, S):
            rows_t += pipelined(b, b + 1 if b + 1 < S else None)
            if (b - args.warmup) % 4 == 3:
                log("step %d/%d  %.2fs" % (b - args.warmup + 1, args.steps, time.perf_counter() - t0))
    elif async_fire:
        # the watermark step returns while its fire runs (fwa_advance_watermark_async); the fired rows are taken
        # after the next batch was handed over, so the host's work for batch b+1 overlaps the fire of batch b
        for b in range(args.warmup, S):
            dropped += push(b)
            if b > args.warmup:
                rows_t += eng.fired_output_raw().n_rows
            eng.advance_watermark_async(wms[b])
            if (b - args.warmup) % 4 == 3:
                log("step %d/%d  %.2fs" % (b - args.warmup + 1, args.steps, time.perf_counter() - t0))
        rows_t += eng.fired_output_raw().n_rows
    else:
        for b in range(args.warmup, S):
            dropped += push(b)
            rows_t += fire(b)
            if (b - args.warmup) % 4 == 3:
                log("step %d/%d  %.2fs" % (b - args.warmup + 1, args.steps, time.perf_counter() - t0))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        rdev = dev if backend == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        rr = torch.tensor([rows_t], dtype=torch.int64, device=rdev)
        dist.all_reduce(rr)
        rows_all = int(rr.item())
    else:
        rows_all = rows_t
    st = eng.stats()
    recs_timed = args.steps * B * world
    value = recs_timed / elapsed

    # live roofline of the dominant kernel (ingest), HIP events on the engine's stream
    ingest_s = st.ingest_ms / 1e3
    rec_bytes = 28 if fp else 24                      # key + ts + val(s), read once; C5: f32 + f64
    alg_bytes_ingest = rec_bytes * st.ingest_records
    achieved = alg_bytes_ingest / ingest_s / 1e9 if ingest_s > 0 else 0.0
    row_bytes = 24 + 8 * len(aggs)                     # key, start, end + one 8 B column per aggregate
    e2e_bytes = rec_bytes * recs_timed + row_bytes * rows_all   # whole-job algorithmic bytes incl. emitted rows
    # HBM traffic per ingest launch (Phase P + Phase A) from the committed rocprofv3 PMC passes of this
    # same workload (counters need their own runs: tools/gpu_pmc.sh); null for other shapes
    traffic, traffic_src, traffic_bounds = None, None, None
    for tag in ("r06", "r05", "r04", "r03", "r02"):
        pmc_path = os.path.join(ROOT, "profiles", "%s_pmc_%s.json" % (tag, args.config))
        if world != 1 or not os.path.exists(pmc_path):
            continue
        pmc = json.load(open(pmc_path))
        if pmc["config"]["batch"] == B:
            traffic = pmc["ingest_bytes_per_launch"]
            traffic_bounds = pmc.get("ingest_bytes_per_launch_bounds")
            traffic_src = ("profiles/%s_pmc_%s.json (rocprofv3 FETCH_SIZE + WRITE_SIZE of the ingest kernels per timed "
                           "step, tools/gpu_pmc_all.sh; FETCH_SIZE x2 %s)"
                           % (tag, args.config, "for the wide streaming readers only, raw / all-x2 bounds beside"
                              if traffic_bounds else "for every kernel"))
        break
    if args.config == "c3":
        metric = "records/sec aggregated (C3: HOP 60s/1s, Zipf(1.1) keys over %d items)" % args.keys
        workload = ("C3: Table HOP 60s/1s (1s slices) COUNT+SUM(long), Zipf(1.1) over %d keys, %d records/GPU "
                    "(%d batches of %d), D=%dms" % (args.keys, args.steps * B, args.steps, B, args.delay_ms))
    elif args.config == "c4":
        metric = "records/sec aggregated (C4: %dM-key tumbling SUM, maxParallelism 128)" % (args.keys // 1_000_000)
        workload = ("C4: event-time tumbling %ds COUNT+SUM(long), %d uniform keys, %d records/GPU "
                    "(%d batches of %d), D=%dms" % (args.window_ms // 1000, args.keys, args.steps * B,
                                                    args.steps, B, args.delay_ms))
    elif args.config == "reduce":
        op = "sum(1)" if args.reduce_op == "sum" else "maxBy(1)"
        metric = "records/sec aggregated (DataStream reduce: WindowedStream.%s, 1M-key tumbling)" % op
        workload = ("reduce: event-time tumbling %ds WindowedStream.%s over Tuple3<Long,Long,Long> (f0 key, f1 "
                    "reduced, f2 = ts of the selected element), %d uniform keys, %d records/GPU (%d batches of %d), "
                    "D=%dms" % (args.window_ms // 1000, op, args.keys, args.steps * B, args.steps, B, args.delay_ms))
    elif fp:
        kind = "Table TUMBLE %ds TVF" % (args.window_ms // 1000) if args.config == "c5" else "DataStream SESSION gap 5s"
        metric = "records/sec aggregated (C5: %s, COUNT/SUM/AVG(double)/MAX(float,double))" % kind
        workload = ("C5: %s, COUNT, SUM(d), AVG(d), MAX(f), MAX(d) over f32/f64 in [0,1), %d uniform keys, "
                    "%d records/GPU (%d batches of %d), D=%dms" % (kind, args.keys, args.steps * B, args.steps, B,
                                                                   args.delay_ms))
    else:
        metric = "records/sec aggregated (1M-key tumbling SUM)"
        workload = ("C2: event-time tumbling %ds COUNT+SUM(long), %d uniform keys, %d records/GPU "
                    "(%d batches of %d), D=%dms" % (args.window_ms // 1000, args.keys, args.steps * B,
                                                    args.steps, B, args.delay_ms))
    xname = "RCCL" if backend == "nccl" else backend + " (rehearsal: blocks staged through the host)"
    out = {
        "metric": metric,
        "value": value,
        "unit": "records/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32+f64" if fp else "int64",
        "data": "synthetic (splitmix64 counter-based stream, SURVEY.md §8(d)), generated in HBM",
        "config": {
            "workload": workload,
            "records_per_gpu_timed": args.steps * B, "keys": args.keys, "batch": B,
            "window_ms": args.window_ms, "parallelism": "key-group dp%d" % world,
            "exchange": ("two-phase partials (local pre-aggregation, fwa_drain_route per-subtask blocks, %s "
                         "all_to_all, owner fwa_fire_partials)" % xname if args.exchange == "partials"
                         else "raw records (%s all_to_all)" % xname) if world > 1 else "none",
        },
        "roofline": {
            "bound": "hbm", "kernel": ingest_kernels(args, eng),
            "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic, "traffic_unit": "bytes per launch",
            "traffic_source": traffic_src, "traffic_bounds": traffic_bounds, "alg_bytes_per_launch": rec_bytes * B,
            "alg_bytes_per_record": rec_bytes, "launches": st.ingest_launches,
            "avg_launch_ms": st.ingest_ms / max(1, st.ingest_launches),
        },
        # the fire kernels' own roofline (per step: emitted rows x row bytes over the fire device time, HIP
        # events on the engine stream); for C4 (record lists) the fire is the larger device cost of a step
        "roofline_fire": {
            "bound": "hbm", "kernel": fire_kernels(args, eng),
            "achieved": (row_bytes * st.fire_rows / (st.fire_ms / 1e3) / 1e9) if st.fire_ms > 0 else 0.0,
            "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": (row_bytes * st.fire_rows / (st.fire_ms / 1e3) / 1e9 / HBM_PEAK_GBPS) if st.fire_ms > 0 else 0.0,
            "alg_bytes_per_launch": row_bytes * st.fire_rows / max(1, args.steps), "alg_bytes_per_row": row_bytes,
            "ms_per_step": st.fire_ms / max(1, args.steps),
        },
        # push + fire device time of a step against the step's algorithmic bytes (input + emitted rows)
        "roofline_step": {
            "achieved": ((alg_bytes_ingest + row_bytes * st.fire_rows) / ((st.ingest_ms + st.fire_ms) / 1e3) / 1e9)
            if st.ingest_ms + st.fire_ms > 0 else 0.0,
            "frac": ((alg_bytes_ingest + row_bytes * st.fire_rows) / ((st.ingest_ms + st.fire_ms) / 1e3) / 1e9
                     / HBM_PEAK_GBPS) if st.ingest_ms + st.fire_ms > 0 else 0.0,
            "device_ms_per_step": (st.ingest_ms + st.fire_ms) / max(1, args.steps),
        },
        "end_to_end_hbm_frac": e2e_bytes / elapsed / 1e9 / HBM_PEAK_GBPS / world,
        "fire": {"launches": st.fire_launches, "ms": st.fire_ms, "rows": st.fire_rows},
        "ingest_split_ms": {"partition": st.partition_ms, "combine": st.combine_ms, "total": st.ingest_ms},
        "rows_emitted": rows_all,
        "late_dropped": sum(x.stats().late_dropped for x in engines) if args.exchange == "partials" or world == 1 else dropped,
    }
    out["roofline"]["replay_records"] = st.replay_records
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "c2":
        out["cpu_baseline"] = cpu_baseline(args, cfg_kw)
    if rank == 0 and world == 1 and not args.no_pcie and args.config == "c2":
        out["pcie_inclusive"] = pcie_leg(args, cfg_kw, keys, ts, vals, wms, dev)
    if rank == 0 and world == 1 and not args.no_wide and args.config == "c2":
        out["wide_keys"] = wide_keys_leg(args, cfg_kw, keys, ts, vals, wms, dev)
    if rank == 0 and world == 1 and not args.no_wire and args.config == "c2":
        out["wire_input"] = wire_leg(args, cfg_kw, keys, ts, vals, wms, dev)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def ingest_kernels(args, eng):
    """Names of the kernels whose device time `roofline.achieved` divides by (HIP events around them)."""
    if args.config == "c5s":
        return ("s5_hist+s5_colscan+scan+s5_part+s5_resolve+s4_sess_count/scatter+s4_group+s4_compact (cell "
                "pre-aggregation, hash route; sess3_* sort-based cells or sess2_* when a push leaves its range)")
    if eng.record_lists:
        return "sp_range_kernel+sp_hist_kernel+sp_scan_kernel+sp_scatter_kernel (record lists)"
    if args.config == "reduce":
        return ("partition3_kernel+combine3_kernel+red_iota_payload_kernel (two-phase ingest with the record-index "
                "accumulator in narrow entries, the index derived in partition3, then the payload pass)")
    return "partition3_kernel+combine3_kernel" if eng.stats().partition_ms > 0 else "ingest_kernel"


def fire_kernels(args, eng):
    """Names of the kernels whose device time `roofline_fire` divides by."""
    if args.config == "c5s":
        return "sess2_fire_kernel"
    if eng.record_lists:
        return "sp_refine_kernel+sp_agg_kernel (record lists)"
    if args.config == "reduce":
        return "red_fire_kernel"
    return "fire_slide_kernel" if args.config == "c3" else "fire_kernel"


def host_cpus():
    """CPUs this process may run on (affinity, capped by a cgroup v2 quota when one is set) and the model."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return n, quota, os.cpu_count(), model


def cpu_baseline(args, cfg_kw):
    """The oracle's multi-threaded restatement of the heap WindowOperator pipeline (keyBy partition +
    one operator instance per thread owning a key-group range), timed on this host's cores."""
    from flink_amd import _abi as A
    from oracle import oracle as O
    avail, quota, nproc, model = host_cpus()
    threads = args.cpu_threads or (min(avail, quota) if quota else avail)
    n = args.cpu_sample
    cfg = A.make_config(window_kind="TUMBLE", semantics="DATASTREAM", size_ms=args.window_ms,
                        aggs=[("COUNT", 0), ("SUM_I64", 0)])
    p = A.GenParams(seed_k=0x5eed0001, seed_t=0x5eed0002, seed_v=0x5eed0003, first_index=0,
                    total_records=C2_RECORDS, num_keys=args.keys, t0_ms=1_700_000_000_000, span_ms=C2_SPAN_MS,
                    max_delay_ms=args.delay_ms, key_dist=0, val_kind=0)
    log("cpu baseline: %d records, %d threads" % (n, threads))
    secs, rows, _ = O.bench_pipeline(cfg, p, n, min(args.batch, n), threads)
    return {"value": n / secs, "unit": "records/s", "cores": threads, "kind": "port",
            "host": {"cpu_model": model, "nproc": nproc, "affinity_cpus": avail, "cgroup_cpu_quota": quota},
            "sample": "first %d records of the C2 stream (%d batches of %d, %d s of event time), oracle "
                      "WindowOperator restatement, %d threads each owning a key-group range (keyBy partition "
                      "untimed); %.2f s" % (n, (n + args.batch - 1) // args.batch, args.batch, n // 1_000_000,
                                            threads, secs)}


def pcie_leg(args, cfg_kw, keys, ts, vals, wms, dev):
    """Secondary number: the same C2 step with the batch handed over in host pinned
    memory (fwa_push without FWA_PUSH_DEVICE_PTRS: the engine stages it over PCIe), timed per batch."""
    import torch
    from flink_amd import _abi as A
    from flink_amd import engine as E
    B = args.batch
    nb = min(args.pcie_batches, args.warmup + args.steps)
    hk = torch.empty(nb * B, dtype=torch.int64, pin_memory=True)
    ht = torch.empty_like(hk, pin_memory=True)
    hv = torch.empty_like(hk, pin_memory=True)
    hk.copy_(keys[:nb * B])
    ht.copy_(ts[:nb * B])
    hv.copy_(vals[:nb * B])
    torch.cuda.synchronize()
    kw = dict(cfg_kw)
    kw["output_on_device"] = 1
    eng = E.WindowAggregator(A.make_config(**kw))
    nk, nt, nv = hk.numpy(), ht.numpy(), hv.numpy()
    eng.push(nk[:B], nt[:B], [nv[:B]])            # warm-up batch (directory, slots, staging buffer)
    eng.advance_watermark_raw(wms[0])
    t0 = time.perf_counter()
    for b in range(1, nb):
        sl = slice(b * B, (b + 1) * B)
        eng.push(nk[sl], nt[sl], [nv[sl]])
        eng.advance_watermark_raw(wms[b])
    secs = time.perf_counter() - t0
    eng.close()
    return {"value": (nb - 1) * B / secs, "unit": "records/s", "batches_timed": nb - 1,
            "note": "host pinned input columns, H2D staging inside fwa_push, outputs left in HBM"}


def wide_keys_leg(args, cfg_kw, keys, ts, vals, wms, dev):
    """Secondary number: the same C2 step with keys that need 64 bits (each key + 2^40), so the
    combiner's 10-byte narrow bucket entries (COUNT + SUM(BIGINT) with 32-bit keys and values) do not apply and
    every record takes the 18-byte entries of the general path. Inputs in HBM, per-batch push + watermark as in the
    main loop."""
    import torch
    from flink_amd import _abi as A
    from flink_amd import engine as E
    B = args.batch
    nb = min(args.wide_batches, args.warmup + args.steps)
    wk = keys[:nb * B] + (1 << 40)
    eng = E.WindowAggregator(A.make_config(**cfg_kw))
    views = [(wk[b * B:(b + 1) * B], ts[b * B:(b + 1) * B], [vals[b * B:(b + 1) * B]]) for b in range(nb)]
    for b in range(2):                            # warm-up: the first push finds the 64-bit keys (narrow off)
        eng.push(*views[b], sync=False)
        eng.advance_watermark_raw(wms[b])
    eng.reset_timers()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in range(2, nb):
        eng.push(*views[b], sync=False)
        eng.advance_watermark_raw(wms[b])
    torch.cuda.synchronize()
    secs = time.perf_counter() - t0
    st = eng.stats()
    narrow = eng.get_option("narrow_entries")
    eng.close()
    del wk
    return {"value": (nb - 2) * B / secs, "unit": "records/s", "batches_timed": nb - 2,
            "ms_per_step": secs * 1e3 / (nb - 2), "narrow_entries": bool(narrow),
            "ingest_ms_per_step": st.ingest_ms / max(1, st.ingest_launches),
            "note": "keys + 2^40 (64-bit keys): 18-byte bucket entries instead of the 10-byte narrow ones"}


def encode_c2_wire(k, t, v, wm, dev):
    """The C2 batch as a network channel would carry it (bench input, built on the device): every record a
    StreamRecord<Tuple3<Long, Long, Long>>(key, ts, val) with its timestamp -- 4-byte big-endian length 33,
    tag 0, ts, then the three longs (RecordWriter.serializeRecord + StreamElementSerializer.serialize +
    TupleSerializer, SURVEY.md a4: 37 B per record) -- followed by the batch's watermark element."""
    import torch

    def be(x):   # int64 -> 8 big-endian bytes per element
        return x.contiguous().view(torch.uint8).view(-1, 8).flip(1)
    n = k.shape[0]
    rec = torch.empty(n, 37, dtype=torch.uint8, device=dev)
    rec[:, 0:4] = torch.tensor([0, 0, 0, 33], dtype=torch.uint8, device=dev)
    rec[:, 4] = 0
    rec[:, 5:13] = be(t)
    rec[:, 13:21] = be(k)
    rec[:, 21:29] = be(t)
    rec[:, 29:37] = be(v)
    w = torch.tensor([0, 0, 0, 9, 2], dtype=torch.uint8, device=dev)
    wv = be(torch.tensor([wm], dtype=torch.int64, device=dev)).reshape(-1)
    return torch.cat([rec.reshape(-1), w, wv])


def wire_leg(args, cfg_kw, keys, ts, vals, wms, dev):
    """Secondary number: the C2 step fed from network bytes already in HBM --
    fwa_wire_decode (boundary scan + decode into SoA columns) -> fwa_push of the decoded columns -> the
    watermark element -> fwa_advance_watermark. Also the decode kernels' own roofline: 37 B of wire bytes
    read + 24 B of columns written per record (61 B algorithmic), HIP events on the decoder's stream."""
    import torch
    from flink_amd import _abi as A
    from flink_amd import engine as E
    from flink_amd import wire
    B = args.batch
    nb = min(args.wire_batches, args.warmup + args.steps)
    bufs = [encode_c2_wire(keys[b * B:(b + 1) * B], ts[b * B:(b + 1) * B], vals[b * B:(b + 1) * B], wms[b], dev)
            for b in range(nb)]
    torch.cuda.synchronize()
    eng = E.WindowAggregator(A.make_config(**cfg_kw))
    dec = wire.WireDecoder(wire.make_schema(["LONG", "LONG", "LONG"], key_field=0, ts_field=-1, cols=[2],
                                            device=dev.index or 0, max_bytes=bufs[0].numel()))

    def step(b):
        d = dec.decode(bufs[b])
        assert d.n_records == B and d.n_events == 1 and d.evt_pos[0] == B
        eng.push(d.key, d.ts, d.cols)
        return eng.advance_watermark_raw(int(d.evt_val[0][0])).n_rows
    step(0)                                        # warm-up batch
    st0 = dec.stats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in range(1, nb):
        step(b)
    torch.cuda.synchronize()
    secs = time.perf_counter() - t0
    st = dec.stats()
    calls = st.calls - st0.calls
    dms = (st.decode_ms - st0.decode_ms) / calls
    sms = (st.scan_ms - st0.scan_ms) / calls
    alg = 61 * B
    eng.close()
    dec.close()
    return {"value": (nb - 1) * B / secs, "unit": "records/s", "batches_timed": nb - 1,
            "wire_bytes_per_batch": int(bufs[0].numel()),
            "decode": {"kernels": "wire_scan_kernel+wire_compose_kernel+wire_resolve_kernel+wire_decode_kernel",
                       "ms_per_batch": dms, "scan_ms_per_batch": sms, "records_per_s": B / (dms / 1e3),
                       "alg_bytes_per_record": 61, "achieved": alg / (dms / 1e3) / 1e9, "peak": HBM_PEAK_GBPS,
                       "unit": "GB/s", "frac": alg / (dms / 1e3) / 1e9 / HBM_PEAK_GBPS},
            "note": "Tuple3<Long,Long,Long> StreamRecords with timestamps (37 B each) + one watermark element per "
                    "batch, in HBM; decode + push + fire timed per batch, outputs left in HBM"}


if __name__ == "__main__":
    main()
