"""Key-group-partitioned multi-GPU window aggregation: one process per GPU, torch.distributed
(backend "nccl" = RCCL over xGMI on MI355X; "gloo" for the CPU tests).

Reference structure this replaces:
  keyBy shuffle   KeyGroupStreamPartitioner.selectChannel  SJ/runtime/partitioner/KeyGroupStreamPartitioner.java:55-65
                  -> RecordWriter/Netty network stack      RT/io/network/api/writer/RecordWriter.java:104-157
  ownership       computeKeyGroupRangeForOperatorIndex     RT/state/KeyGroupRangeAssignment.java:93-106
  watermark       StatusWatermarkValve: min over input channels  SJ/runtime/watermarkstatus/StatusWatermarkValve.java:192

Rank r owns key groups key_group_range_for_operator(maxP, world, r). Two exchange plans:

* KeyedWindowPipeline (raw records, the DataStream keyBy): each push routes every record to its owner
  (dest = kg * world / maxP, computed on the GPU) with one all_to_all_single of the packed
  (key, ts, values) rows after an all_to_all of the counts; the owner's engine then accumulates.
* TwoPhaseKeyedWindowPipeline (Flink's two-phase window plan, TwoStageOptimizedWindowAggregateRule
  .java:88-103): every rank pre-aggregates its own source records per (key, slice) in a local engine
  (LocalSlicingWindowAggOperator.java:111-131); at each watermark the complete slices' partial
  accumulators are drained, exchanged by key group in one all_to_all_single, and merged into the
  owner's engine (GlobalAggCombiner.java:77-110), which fires. With 1M keys this ships one 32-40 B
  partial per (key, slice) instead of one 24 B record per input record.

Each advance_watermark takes the MIN over ranks (the valve), then fires locally. No other collective
is on the data path.
"""
import contextlib

import numpy as np
import torch
import torch.distributed as dist

from . import _abi as A
from .keygroups import key_group_range_for_operator


def choose_exchange(cfg_kw):
    """The keyBy plan for a configuration: "partials" (two-phase, TwoStageOptimizedWindowAggregateRule) unless the key
    space is so large that a step's (key, slice) partials barely outnumber its records -- the engine's record-list
    regime (key_capacity >= 2^25, FWA_CFG_RECORD_LISTS; C4's 1e8 keys: ~1 record per key and window) -- where shipping
    partial rows (32-40 B) instead of records (24 B) would grow the exchange: "raw"."""
    kc = int(cfg_kw.get("key_capacity", 0) or 0)
    return "raw" if kc >= 1 << 25 or cfg_kw.get("record_lists") else "partials"


def owner_key_capacity(key_capacity, n_groups, max_parallelism, margin=1.25, slack=4096):
    """Key capacity of an engine owning n_groups of max_parallelism key groups when the job's key space is
    key_capacity keys: its share (keys spread over key groups by a murmur hash, KeyGroupRangeAssignment
    .assignToKeyGroup) with a margin, so a dense owner's fire scans its share of the key table, not the whole job's
    (the table is 2x the capacity, rounded up to a power of two). Record-list sized key spaces (>= 2^25 keys) keep
    their capacity: it selects that layout (FWA_CFG_RECORD_LISTS). A share that overflows fails loudly (FWA_E_OOM)."""
    kc = int(key_capacity or 0)
    if kc <= 0 or kc >= 1 << 25 or n_groups >= max_parallelism:
        return kc
    share = -(-kc * n_groups // max_parallelism)
    return min(kc, int(share * margin) + slack)


_VALVE_GROUPS = {}


def valve_group(group=None):
    """The process group the watermark valve's MIN-allreduce runs on. Under RCCL it is a gloo group over the same
    ranks, so the valve works on host integers without a device synchronisation (a .item() would wait for every kernel
    queued on the stream). One gloo group per rank set, created on first use and cached for the process: creating it is
    collective over the WHOLE default group (torch.distributed.new_group), so the first pipeline built on a given group
    must be constructed on every rank of the job, including ranks outside `group`; later pipelines reuse it."""
    if dist.get_backend(group) != "nccl":
        return group
    ranks = tuple(dist.get_process_group_ranks(group)) if group is not None else tuple(range(dist.get_world_size()))
    g = _VALVE_GROUPS.get(ranks)
    if g is None:
        g = dist.new_group(ranks=list(ranks), backend="gloo")
        _VALVE_GROUPS[ranks] = g
    return g


def _gpu_router(max_parallelism, world, key_kind):
    from . import engine

    def route(keys):
        _, op = engine.key_groups(keys, max_parallelism, world, key_kind=key_kind, device=keys.device.index or 0)
        return torch.as_tensor(op).to(torch.int64)
    return route


class KeyedWindowPipeline:
    """One Flink subtask per rank: keyBy exchange + a window engine owning this rank's key groups."""

    def __init__(self, rank, world, group=None, engine_factory=None, router=None, owner_capacity="share", **cfg_kw):
        """owner_capacity: "share" sizes the owning engine's key table to its key groups' share of key_capacity
        (owner_key_capacity), "full" keeps the job's key_capacity, an int sets it."""
        self.rank, self.world, self.group = rank, world, group
        maxp = cfg_kw.get("max_parallelism", 128)
        kg0, kg1 = key_group_range_for_operator(maxp, world, rank)
        okw = dict(cfg_kw)
        if owner_capacity == "share":
            if not cfg_kw.get("record_lists") and cfg_kw.get("key_capacity"):
                okw["key_capacity"] = owner_key_capacity(cfg_kw.get("key_capacity", 0), kg1 - kg0 + 1, maxp)
        elif owner_capacity != "full":
            okw["key_capacity"] = int(owner_capacity)
        self.cfg = A.make_config(kg_start=kg0, kg_end=kg1, **okw)
        if engine_factory is None:
            from .engine import WindowAggregator
            engine_factory = WindowAggregator
        self.engine = engine_factory(self.cfg)
        self.route = router or _gpu_router(maxp, world, self.cfg.key_kind)
        self.route_on_gpu = router is None          # a custom router (tests) keeps the torch grouping
        self.names = A.agg_names(self.cfg)
        self.exchanged = 0
        self.wm_group = valve_group(group)       # host-side MIN valve (gloo under RCCL; see valve_group)
        self._xstream = None

    def _exchange_stream(self, t):
        """The exchange's own torch stream for CUDA batches: routing, the all-to-all and the engine's read of the
        received rows are ordered on the device (the engine waits for this stream through fwa_set_input_stream), so
        no step waits on the host for torch's default stream, which the engine's stream cannot wait on."""
        if not t.is_cuda:
            return contextlib.nullcontext()
        if self._xstream is None:
            self._xstream = torch.cuda.Stream(device=t.device)
        self._xstream.wait_stream(torch.cuda.current_stream(t.device))   # the batch's producers
        return torch.cuda.stream(self._xstream)

    def _a2a(self, x, send_splits, recv_splits):
        out = torch.empty(sum(recv_splits), dtype=x.dtype, device=x.device)
        dist.all_to_all_single(out, x, recv_splits, send_splits, group=self.group)
        return out

    def push(self, keys, ts, cols=()):
        """keys/ts/cols: this rank's source records (torch tensors on the rank's device)."""
        cols = list(cols)
        with self._exchange_stream(keys):
            recv = exchange_rows(self, keys, [keys, ts] + cols)
            k, t = recv[:, 0].contiguous(), recv[:, 1].contiguous()
            c = [unpack_col(recv[:, 2 + j], x.dtype) for j, x in enumerate(cols)]
            if k.is_cuda:
                return self.engine.push(k, t, c)
        return self.engine.push(k.numpy(), t.numpy(), [x.numpy() for x in c])

    def global_watermark(self, local_wm):
        """StatusWatermarkValve (StatusWatermarkValve.java:192): the MIN over ranks, on the host (gloo)."""
        w = torch.tensor([int(local_wm)], dtype=torch.int64)
        dist.all_reduce(w, op=dist.ReduceOp.MIN, group=self.wm_group)
        return int(w[0])

    def advance_watermark(self, local_wm, device_output=False):
        wm = self.global_watermark(local_wm)
        if device_output:
            return self.engine.advance_watermark_device(wm)
        return self.engine.advance_watermark(wm)

    def close(self):
        self.engine.close()


def unpack_col(cell, dtype):
    """Inverse of exchange_rows' packing for one column."""
    if dtype.itemsize == 8:
        return cell.contiguous().view(dtype)
    return cell.to(torch.int32).view(dtype).contiguous()


def route_rows(pipe, keys, cols):
    """The send side of the keyBy exchange: rows packed by destination (int64 [n, m]) and per-destination counts.
    Device batches use the HIP counting sort (fwa_route_rows); host tensors (the gloo tests) the same stable
    grouping in torch."""
    n = int(keys.shape[0])
    if keys.is_cuda and pipe.route_on_gpu:
        from . import engine
        return engine.route_rows(keys, [c.contiguous() for c in cols], pipe.cfg.max_parallelism, pipe.world,
                                 key_kind=pipe.cfg.key_kind)
    dest = pipe.route(keys)
    packed = torch.empty((n, len(cols)), dtype=torch.int64, device=keys.device)
    for j, x in enumerate(cols):
        packed[:, j] = x.view(torch.int64) if x.dtype.itemsize == 8 else x.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    if pipe.world > 1:
        order = torch.argsort(dest, stable=True)
        packed = packed[order]
    return packed, torch.bincount(dest, minlength=pipe.world)


def host_counts(counts):
    """The route's per-destination row counts on the host: one copy into pinned memory and one wait on the stream
    that computed them (all_to_all_single needs host split sizes; this is the push's only host wait)."""
    if not counts.is_cuda:
        return counts
    h = torch.empty(counts.shape, dtype=counts.dtype, pin_memory=True)
    h.copy_(counts, non_blocking=True)
    torch.cuda.current_stream(counts.device).synchronize()
    return h


def send_rows(pipe, packed, counts):
    """The split sizes travel on the host (the valve's gloo group, as send_parts), the packed rows in one
    all_to_all_single (RCCL over xGMI): no collective kernel and no device read for the counts matrix."""
    sc = host_counts(counts)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=pipe.wm_group)
    send = sc.tolist()
    recv = rc.tolist()
    out = torch.empty((sum(recv), packed.shape[1]), dtype=torch.int64, device=packed.device)
    dist.all_to_all_single(out, packed, recv, send, group=pipe.group)
    pipe.exchanged += int(sum(send)) - int(send[pipe.rank])
    return out


def send_parts(pipe, parts, counts, m):
    """The exchange of fwa_drain_route's per-destination row blocks: the split sizes are the drain's host counts,
    exchanged on the host (the valve's gloo group: no device read), then one all_to_all of the blocks (RCCL)."""
    sc = torch.tensor(counts, dtype=torch.int64)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=pipe.wm_group)
    recv = rc.tolist()
    if dist.get_backend(pipe.group) == "nccl":
        out = torch.empty((sum(recv), m), dtype=torch.int64, device=parts[0].device)
        dist.all_to_all(list(out.split(recv)), [p.contiguous() for p in parts], group=pipe.group)
    else:                                              # gloo rehearsal: host staging of the device blocks
        host = torch.empty((sum(recv), m), dtype=torch.int64)
        dist.all_to_all_single(host, torch.cat(parts).cpu(), recv, counts, group=pipe.group)
        out = host.to(parts[0].device)
    pipe.exchanged += sum(counts) - counts[pipe.rank]
    return out


def exchange_rows(pipe, keys, cols):
    """keyBy exchange of a row set: route by key group, pack the columns into one int64 [n, m] tensor grouped by
    destination, exchange (RCCL over xGMI). Returns the received rows (int64 [n_recv, m]; 4-byte columns travel
    zero-extended in their 8-byte cell)."""
    packed, counts = route_rows(pipe, keys, cols)
    return send_rows(pipe, packed, counts)


class TwoPhaseKeyedWindowPipeline(KeyedWindowPipeline):
    """One Flink subtask per rank in the two-phase plan: a local pre-aggregating engine over this
    rank's source records (all key groups), then the partial-accumulator keyBy exchange into the
    engine owning this rank's key groups. Same push / advance_watermark surface as
    KeyedWindowPipeline; pushes involve no collective."""

    def __init__(self, rank, world, group=None, engine_factory=None, router=None, local_factory=None,
                 owner_capacity="share", routed=None, **cfg_kw):
        """routed: the drain writes the exchange's per-subtask blocks itself (fwa_drain_route); default under RCCL,
        True forces it on a gloo group (rehearsals on one GPU: the blocks are staged through the host)."""
        super().__init__(rank, world, group=group, engine_factory=engine_factory, router=router,
                         owner_capacity=owner_capacity, **cfg_kw)
        lkw = dict(cfg_kw)
        if routed is None:
            routed = dist.get_backend(group) == "nccl"
        lkw["output_on_device"] = 1 if (routed or dist.get_backend(group) == "nccl") else 0
        self.local_cfg = A.make_config(**lkw)           # the pre-aggregator sees every key group
        if local_factory is None:
            from .engine import WindowAggregator
            local_factory = WindowAggregator
        self.local = local_factory(self.local_cfg)
        self.partials_sent = 0
        # the drain writes the send layout itself (fwa_drain_route) when the local engine is a device handle
        self.routed_drain = bool(routed) and hasattr(self.local, "drain_route")

    def push(self, keys, ts, cols=()):
        if keys.is_cuda:
            return self.local.push(keys, ts, list(cols), sync=False)
        return self.local.push(keys.numpy(), ts.numpy(), [x.numpy() for x in cols])

    def advance_watermark(self, local_wm, device_output=False, then_push=None):
        """then_push: (keys, ts, cols) of this rank's next batch, pushed into the local pre-aggregator as soon as the
        drained partials are routed -- its ingest then runs while the exchange, the owner's merge and the fire of
        this watermark proceed (software pipelining across steps; each engine still sees its own calls in stream
        order: drain(wm), push(next) on the local one, merge(wm), fire(wm) on the owner)."""
        wm = self.global_watermark(local_wm)
        if self._xstream is not None and hasattr(self.local, "order_after"):
            # the previous watermark's exchange (its own stream) may still read the blocks / columns the last drain
            # returned: this drain rewrites them only after everything queued there
            self.local.order_after(self._xstream)
        if self.routed_drain:
            try:
                parts, counts, m = self.local.drain_route(wm, self.world)
            except RuntimeError as ex:                  # FWA_E_UNSUPPORTED (e.g. record lists): drain, then route
                if getattr(ex, "code", None) != -7:
                    raise
                self.routed_drain = False
            else:
                return self._send_routed_and_fire(wm, parts, counts, m, device_output, then_push)
        p = self.local.drain_partials(wm)
        # a COUNT(*) aggregate's accumulator repeats the row count: it is not shipped (rebuilt on arrival)
        ship = [j for j, name in enumerate(self.names) if name != "COUNT"]
        nh = sum(1 for f in p if f.startswith("hidden"))  # SQL NULLs: the hidden non-NULL counters travel too
        cols = [p["key"], p["slice_start"], p["count"]] + [p["acc%d" % j] for j in ship] + \
            [p["hidden%d" % h] for h in range(nh)]
        cols = [c if isinstance(c, torch.Tensor) else torch.from_numpy(c) for c in cols]
        with self._exchange_stream(cols[0]):
            return self._exchange_and_fire(wm, cols, ship, nh, device_output, then_push)

    def _send_routed_and_fire(self, wm, parts, counts, m, device_output, then_push):
        ship = [j for j, name in enumerate(self.names) if name != "COUNT"]
        nh = m - 3 - len(ship)
        with self._exchange_stream(parts[0]):
            if then_push is not None:
                self.push(*then_push)
            recv = send_parts(self, parts, counts, m)
            self.partials_sent += sum(counts)
            cells = [2 if name == "COUNT" else 3 + ship.index(j) for j, name in enumerate(self.names)] + \
                [3 + len(ship) + h for h in range(nh)]
            return self.engine.fire_partials(recv, cells, wm, device_output=device_output)

    def _exchange_and_fire(self, wm, cols, ship, nh, device_output, then_push):
        packed, counts = route_rows(self, cols[0], cols)    # done with the drained buffers from here on
        if then_push is not None:
            self.push(*then_push)
        recv = send_rows(self, packed, counts)
        self.partials_sent += int(cols[0].shape[0])
        if recv.is_cuda and hasattr(self.engine, "fire_partials"):
            # merge + fire straight from the receive buffer (fwa_fire_partials: on chip for TUMBLE windows without
            # lateness, else push_partials + advance_watermark inside the call)
            cells = [2 if name == "COUNT" else 3 + ship.index(j) for j, name in enumerate(self.names)] + \
                [3 + len(ship) + h for h in range(nh)]
            return self.engine.fire_partials(recv, cells, wm, device_output=device_output)
        if recv.is_cuda:
            from . import engine
            col = engine.unpack_rows(recv)
        else:
            col = [recv[:, j].contiguous() for j in range(recv.shape[1])]
        if not recv.is_cuda:
            col = [c.numpy() for c in col]
        accs, k = [], 3
        for name in self.names:
            if name == "COUNT":
                accs.append(col[2])
            else:
                accs.append(col[k])
                k += 1
        self.engine.push_partials(col[0], col[1], col[2], accs, hidden=col[k:k + nh])
        if device_output:
            return self.engine.advance_watermark_device(wm)
        return self.engine.advance_watermark(wm)

    def close(self):
        self.local.close()
        super().close()


def merge_rows(parts, names):
    """Concatenate fired-row dicts (e.g. gathered from all ranks) into one dict of numpy columns."""
    out = {}
    for f in ["key", "win_start", "win_end"] + ["agg%d" % j for j in range(len(names))]:
        out[f] = np.concatenate([p[f] for p in parts]) if parts else np.zeros(0)
    return out
