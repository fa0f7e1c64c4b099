"""ctypes binding of libflink_amd.so (the HIP engine behind include/flink_amd.h).

`WindowAggregator` is the thin host handle the operator facades (flink_amd.operators) sit on. Inputs
may be numpy arrays (host; staged by the engine) or torch CUDA tensors (device pointers, zero copy).
There is no CPU fallback: if the HIP library is missing this module raises at import/first use.
"""
import ctypes as C
import os

import numpy as np

from . import _abi as A

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libflink_amd.so")
_LIB = None


class EngineError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s: %s" % (A.STATUS.get(code, code), msg))
        self.code = code


class Blob(C.Structure):
    """fwa_blob (include/flink_amd.h): engine-allocated snapshot buffer."""
    _fields_ = [("data", C.c_void_p), ("size", C.c_int64)]


def lib():
    """Load libflink_amd.so (built by `make -C flink_amd/csrc` / __graft_entry__.build())."""
    global _LIB
    if _LIB is not None:
        return _LIB
    _init_torch_runtime_first()
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("libflink_amd.so not built (%s): run `make -C flink_amd/csrc`; "
                           "there is no CPU fallback for the engine" % LIB_PATH)
    L = C.CDLL(LIB_PATH)
    A.bind_common(L, "fwa_")
    L.fwa_push.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64,
                           C.c_int32, C.POINTER(C.c_int64)]
    L.fwa_push.restype = C.c_int
    L.fwa_push_nullable.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_int64, C.c_int32, C.POINTER(C.c_int64)]
    L.fwa_push_nullable.restype = C.c_int
    L.fwa_drain_partials.argtypes = [C.c_void_p, C.c_int64, C.POINTER(A.Partials)]
    L.fwa_drain_partials.restype = C.c_int
    L.fwa_push_partials.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64,
                                    C.c_int32, C.POINTER(C.c_int64)]
    L.fwa_push_partials.restype = C.c_int
    L.fwa_fire_partials.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.POINTER(C.c_int32), C.c_int64,
                                    C.c_int32, C.POINTER(A.Out), C.POINTER(C.c_int64)]
    L.fwa_fire_partials.restype = C.c_int
    L.fwa_drain_route.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.POINTER(A.Routed)]
    L.fwa_drain_route.restype = C.c_int
    L.fwa_snapshot.argtypes = [C.c_void_p, C.POINTER(Blob)]
    L.fwa_snapshot.restype = C.c_int
    L.fwa_blob_free.argtypes = [C.POINTER(Blob)]
    L.fwa_blob_free.restype = None
    L.fwa_restore.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_int64), C.c_int32]
    L.fwa_restore.restype = C.c_int
    L.fwa_snapshot_heap.argtypes = [C.c_void_p, C.POINTER(Blob), C.c_void_p, C.POINTER(C.c_int64)]
    L.fwa_snapshot_heap.restype = C.c_int
    L.fwa_restore_heap.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                   C.c_int32]
    L.fwa_restore_heap.restype = C.c_int
    L.fwa_snapshot_heap_keys.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(Blob), C.c_void_p, C.POINTER(C.c_int64)]
    L.fwa_snapshot_heap_keys.restype = C.c_int
    L.fwa_restore_heap_keys.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_int64),
                                        C.POINTER(C.c_int64), C.c_int32]
    L.fwa_restore_heap_keys.restype = C.c_int
    L.fwa_flush.argtypes = [C.c_void_p]
    L.fwa_get_config.argtypes = [C.c_void_p, C.POINTER(A.Config)]
    L.fwa_get_config.restype = C.c_int
    L.fwa_flush.restype = C.c_int
    L.fwa_version.restype = C.c_char_p
    L.fwa_set_input_stream.argtypes = [C.c_void_p, C.c_void_p]
    L.fwa_set_input_stream.restype = C.c_int
    L.fwa_late_records.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]
    L.fwa_late_records.restype = C.c_int
    L.fwa_reset_timers.argtypes = [C.c_void_p]
    L.fwa_reset_timers.restype = C.c_int
    L.fwa_key_groups.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_int32,
                                 C.c_void_p, C.c_void_p, C.c_int32, C.c_int32]
    L.fwa_key_groups.restype = C.c_int
    L.fwa_route_rows.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_void_p,
                                 C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
    L.fwa_route_rows.restype = C.c_int
    L.fwa_unpack_rows.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p]
    L.fwa_unpack_rows.restype = C.c_int
    L.fwa_generate.argtypes = [C.POINTER(A.GenParams), C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                               C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
    L.fwa_generate.restype = C.c_int
    L.fwa_set_option.argtypes = [C.c_void_p, C.c_int32, C.c_int64]
    L.fwa_set_option.restype = C.c_int
    L.fwa_get_option.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_int64)]
    L.fwa_get_option.restype = C.c_int
    L.fwa_advance_watermark_async.argtypes = [C.c_void_p, C.c_int64]
    L.fwa_advance_watermark_async.restype = C.c_int
    L.fwa_fired_output.argtypes = [C.c_void_p, C.POINTER(A.Out)]
    L.fwa_fired_output.restype = C.c_int
    L.fwa_stats_size.argtypes = []
    L.fwa_stats_size.restype = C.c_int64
    if L.fwa_stats_size() != C.sizeof(A.Stats):       # the library and this binding disagree on fwa_stats
        raise RuntimeError("fwa_stats is %d bytes in %s, %d in flink_amd._abi" % (L.fwa_stats_size(), LIB_PATH,
                                                                                 C.sizeof(A.Stats)))
    _LIB = L
    return L


def _init_torch_runtime_first():
    """torch bundles its own HIP runtime; if libflink_amd.so's (/opt/rocm) runtime initialises first,
    torch's later sees no GPU. Initialise torch's runtime first when torch and a GPU are present."""
    try:
        import torch
        if torch.cuda.device_count() > 0:
            torch.cuda.init()
    except Exception:
        pass


def _is_torch_cuda(x):
    return type(x).__module__.startswith("torch") and getattr(x, "is_cuda", False)


def _ptr(x):
    if x is None:
        return None
    if _is_torch_cuda(x):
        return C.c_void_p(x.data_ptr())
    return x.ctypes.data_as(C.c_void_p)


def _same_side(device, **named):
    """A batch is all device tensors or all host arrays: a host pointer handed over as a device one (e.g. numpy NULL
    flags beside CUDA key columns) would be dereferenced by a kernel."""
    for name, xs in named.items():
        for x in (xs if isinstance(xs, (list, tuple)) else [xs]):
            if x is not None and _is_torch_cuda(x) != device:
                raise ValueError("%s: %s columns beside %s keys" % (name, "CUDA" if not device else "host",
                                                                     "CUDA" if device else "host"))


def _check(rc, h=None, what=""):
    if rc:
        msg = lib().fwa_last_error(h).decode() if h else what
        raise EngineError(rc, msg or what)


# fwa_set_option (include/flink_amd.h enum fwa_option): per-handle tuning / test options
OPTIONS = {"skew_merge": 1, "window_passes": 2, "narrow_entries": 3, "session_cells": 4, "out_min_rows": 5,
           "partials_one_pass": 6, "sp_table": 7, "sp_fmax": 8, "sp_budget": 9, "profile": 10,
           "session_path": 11, "ingest_variant": 12, "slide_carried": 13, "fire_partials": 14, "dec_wrap_null": 15}
# options applied to every new handle of this process before its own (test tooling sets these, e.g.
# tests/forced_modes_check.py); empty in production
DEFAULT_OPTIONS = {}


class WindowAggregator:
    """One engine handle = one Flink subtask's window operator state (single-threaded)."""

    def __init__(self, cfg, options=None):
        self.cfg = cfg
        self.names = A.agg_names(cfg)
        self.h = C.c_void_p()
        self._inflight = None     # inputs of an FWA_PUSH_ASYNC push, kept alive until the next call settles it
        self._in_stream = None
        rc = lib().fwa_create(C.byref(cfg), C.byref(self.h))
        if rc:
            raise EngineError(rc, "fwa_create")
        for name, value in DEFAULT_OPTIONS.items():    # where they apply to this handle's state layout
            opt = OPTIONS[name] if name in OPTIONS else int(name)
            rc = lib().fwa_set_option(self.h, opt, int(value))
            if rc and rc != -7:                        # FWA_E_UNSUPPORTED: not this layout
                _check(rc, self.h)
        for name, value in (options or {}).items():
            self.set_option(name, value)

    def set_option(self, name, value):
        """fwa_set_option: name from OPTIONS (or the enum value), value -1 adaptive / 0 never / 1 always, or a size."""
        opt = OPTIONS[name] if name in OPTIONS else int(name)
        rc = lib().fwa_set_option(self.h, opt, int(value))
        self._settled()
        _check(rc, self.h)

    def _order_after_producer(self, x):
        """Device inputs come from torch's current stream: make the engine's stream wait for it. torch's legacy
        default stream has no handle the engine's (non-blocking) stream can wait on -- a NULL input stream means
        "the inputs are complete" (fwa_set_input_stream) -- so work still pending there is waited for on the host:
        without it a push read columns the keyBy exchange had not finished writing (the stream-ordered
        fwa_route_rows / fwa_unpack_rows keep no host synchronisation of their own)."""
        import torch
        cs = torch.cuda.current_stream(x.device)
        s = cs.cuda_stream
        if s == 0 and not cs.query():
            cs.synchronize()
        if s != self._in_stream:
            _check(lib().fwa_set_input_stream(self.h, C.c_void_p(s)), self.h)
            self._in_stream = s

    def order_after(self, stream):
        """fwa_set_input_stream(stream): the handle's next push or drain waits for everything enqueued on the torch
        stream `stream` by then (e.g. an exchange still reading the buffers the previous drain returned)."""
        s = stream.cuda_stream
        if s != self._in_stream:
            _check(lib().fwa_set_input_stream(self.h, C.c_void_p(s)), self.h)
            self._in_stream = s

    def _settled(self):
        """Called after every entry point that settles a pending async push."""
        self._inflight = None

    def get_option(self, name):
        """fwa_get_option: the option's effective value (tri-states: 1 if the handle currently takes that path)."""
        opt = OPTIONS[name] if name in OPTIONS else int(name)
        v = C.c_int64(0)
        _check(lib().fwa_get_option(self.h, opt, C.byref(v)), self.h)
        return v.value

    # -- processElement (batched) --
    def push(self, keys, ts, cols=(), key_hash=None, sync=True, nulls=None):
        """Push a columnar batch; returns the number of late records dropped in it.

        sync=False (device inputs only) enqueues the batch and returns 0 at once (FWA_PUSH_ASYNC): the
        batch is settled by the next call on the handle, and the device tensors must stay alive until
        then; late drops are then counted in stats().late_dropped only."""
        device = _is_torch_cuda(keys)
        _same_side(device, ts=ts, cols=list(cols), key_hash=key_hash, nulls=list(nulls or ()))
        if not device:
            keys = np.ascontiguousarray(keys, np.int64)
            ts = np.ascontiguousarray(ts, np.int64)
            cols = [np.ascontiguousarray(c) for c in cols]
            if key_hash is not None:
                key_hash = np.ascontiguousarray(key_hash, np.int32)
        n = int(keys.shape[0])
        arr = (C.c_void_p * max(1, len(cols)))(*[_ptr(c).value for c in cols])
        flags = A.PUSH_DEVICE_PTRS if device else 0
        if device:
            self._order_after_producer(keys)
        if not sync and device:
            flags |= A.PUSH_ASYNC
        dropped = C.c_int64(0)
        if nulls is not None:           # SQL NULL flags per value column (None entries: no NULLs)
            if not device:
                nulls = [None if x is None else np.ascontiguousarray(x, np.uint8) for x in nulls]
            narr = (C.c_void_p * max(1, len(nulls)))(*[None if x is None else _ptr(x).value for x in nulls])
            rc = lib().fwa_push_nullable(self.h, _ptr(keys), _ptr(ts), arr, narr, _ptr(key_hash), n, flags,
                                         C.byref(dropped))
        else:
            rc = lib().fwa_push(self.h, _ptr(keys), _ptr(ts), arr, _ptr(key_hash), n, flags, C.byref(dropped))
        self._settled()
        _check(rc, self.h)
        if flags & A.PUSH_ASYNC:
            self._inflight = (keys, ts, list(cols), key_hash)
        return dropped.value

    # -- processWatermark --
    def advance_watermark_raw(self, wm):
        out = A.Out()
        rc = lib().fwa_advance_watermark(self.h, int(wm), C.byref(out))
        self._settled()
        _check(rc, self.h)
        return out

    def advance_watermark_async(self, wm):
        """fwa_advance_watermark_async: the watermark step without waiting for the fire (rows: fired_output*)."""
        rc = lib().fwa_advance_watermark_async(self.h, int(wm))
        self._settled()
        _check(rc, self.h)

    def fired_output_raw(self):
        """fwa_fired_output: the rows of the last advance_watermark_async (waits for its fire)."""
        out = A.Out()
        _check(lib().fwa_fired_output(self.h, C.byref(out)), self.h)
        return out

    def fired_output(self):
        return self._rows(self.fired_output_raw())

    def advance_watermark(self, wm):
        """Fire every window with maxTimestamp <= wm; returns the fired rows as numpy columns."""
        return self._rows(self.advance_watermark_raw(wm))

    def _rows(self, out):
        n = out.n_rows
        conv = _dev_to_np if out.on_device else _host_to_np
        res = {f: conv(getattr(out, f), n, np.dtype("i8")) for f in ("key", "win_start", "win_end")}
        for j, name in enumerate(self.names):
            if name in A.DEC_KINDS:                    # 16-byte unscaled DECIMAL -> Python ints
                res["agg%d" % j] = A.dec128_values(conv(out.agg[j], 2 * n, np.dtype("i8")))
            else:
                res["agg%d" % j] = conv(out.agg[j], n, np.dtype(A.AGG_RESULT_DTYPE[name]))
            if out.agg_null[j]:
                res["null%d" % j] = conv(out.agg_null[j], n, np.dtype("u1"))
        return res

    def advance_watermark_device(self, wm):
        """Same, but returns zero-copy torch CUDA views of the engine-owned output columns
        (valid until the next call on this handle). Requires output_on_device=1."""
        out = self.advance_watermark_raw(wm)
        n = out.n_rows
        res = {f: dev_view(getattr(out, f), n, np.dtype("i8")) for f in ("key", "win_start", "win_end")}
        for j, name in enumerate(self.names):
            if name in A.DEC_KINDS:                    # int64 [n, 2] (low, high) per row
                res["agg%d" % j] = dev_view(out.agg[j], 2 * n, np.dtype("i8")).view(-1, 2)
            else:
                res["agg%d" % j] = dev_view(out.agg[j], n, np.dtype(A.AGG_RESULT_DTYPE[name]))
        return res

    # -- two-phase aggregation (LocalSlicingWindowAggOperator -> GlobalAggCombiner) --
    def drain_partials(self, wm):
        """Local pre-aggregator watermark step: export the (key, slice) accumulators of every slice
        complete at wm and forward the watermark. Returns dict key/slice_start/count/acc<j> (numpy, or
        zero-copy torch CUDA views valid until the next call when output_on_device=1)."""
        out = A.Partials()
        rc = lib().fwa_drain_partials(self.h, int(wm), C.byref(out))
        self._settled()
        _check(rc, self.h)
        n = out.n
        i8 = np.dtype("i8")
        if out.on_device:
            conv = dev_view
        else:
            conv = _host_to_np
        res = {"key": conv(out.key, n, i8), "slice_start": conv(out.slice_start, n, i8), "count": conv(out.count, n, i8)}
        for j in range(out.num_aggs):
            res["acc%d" % j] = conv(out.acc[j], n, i8)
        for h in range(out.num_hidden):                # nullable handles: hidden non-NULL counters
            res["hidden%d" % h] = conv(out.hidden[h], n, i8)
        return res

    def drain_route(self, wm, parallelism):
        """fwa_drain_route: drain_partials and the keyBy routing in one pass. Returns ([int64 [count_d, cells] torch
        CUDA view per destination d, valid until the next call on this handle], [count_d] host ints, cells)."""
        import torch
        out = A.Routed()
        rc = lib().fwa_drain_route(self.h, int(wm), int(parallelism), C.byref(out))
        self._settled()
        _check(rc, self.h)
        m = out.cells
        dev = torch.device("cuda", self.cfg.device)
        parts = []
        for d in range(parallelism):
            n = out.count[d]
            parts.append(dev_view(out.rows[d], n * m, np.dtype("i8")).view(n, m) if n and out.rows[d]
                         else torch.empty((0, m), dtype=torch.int64, device=dev))
        return parts, [int(out.count[d]) for d in range(parallelism)], m

    def push_partials(self, keys, slice_ts, count, accs, hidden=()):
        """Merge partial accumulators (from drain_partials on a handle with the same window / aggregate
        configuration) into this handle's state; returns the number of late records dropped. `hidden`: the
        hidden non-NULL counter columns of a nullable handle (drain_partials' hidden<h>)."""
        device = _is_torch_cuda(keys)
        _same_side(device, slice_ts=slice_ts, count=count, accs=list(accs), hidden=list(hidden))
        if not device:
            keys = np.ascontiguousarray(keys, np.int64)
            slice_ts = np.ascontiguousarray(slice_ts, np.int64)
            count = np.ascontiguousarray(count, np.int64)
            accs = [np.ascontiguousarray(a).view(np.int64) for a in accs]
            hidden = [np.ascontiguousarray(a, np.int64) for a in hidden]
        nslot = A.FWA_MAX_AGGS + A.FWA_MAX_COLS
        ptrs = [_ptr(a).value for a in accs] + [None] * (self.cfg.num_aggs - len(accs)) + [_ptr(a).value for a in hidden]
        arr = (C.c_void_p * nslot)(*(ptrs + [None] * (nslot - len(ptrs))))
        if device:
            self._order_after_producer(keys)
        dropped = C.c_int64(0)
        rc = lib().fwa_push_partials(self.h, _ptr(keys), _ptr(slice_ts), _ptr(count), arr, int(keys.shape[0]),
                                     A.PUSH_DEVICE_PTRS if device else 0, C.byref(dropped))
        self._settled()
        _check(rc, self.h)
        return dropped.value

    def fire_partials(self, rows, acc_cells, wm, device_output=False):
        """The owner's watermark step over packed partial rows (fwa_fire_partials): the rows of push_partials of the
        rows' cells followed by advance_watermark(wm). rows: int64 [n, m] (torch CUDA: merged and fired on chip
        where the handle allows it; numpy: the two calls), cell 0 key, 1 slice timestamp, 2 COUNT(*); acc_cells[j]:
        the cell of aggregate j's accumulator (user aggregates, then the hidden non-NULL counters; -1 where the
        aggregate keeps none). Returns the fired rows like advance_watermark (advance_watermark_device's torch views
        with device_output=True); late partials are counted in stats().late_dropped."""
        device = _is_torch_cuda(rows)
        if device:
            rows = rows.contiguous()
            self._order_after_producer(rows)
        else:
            rows = np.ascontiguousarray(rows, np.int64)
        n, m = int(rows.shape[0]), int(rows.shape[1]) if rows.ndim == 2 else 0
        nslot = A.FWA_MAX_AGGS + A.FWA_MAX_COLS
        cells = (C.c_int32 * nslot)(*([int(x) for x in acc_cells] + [-1] * (nslot - len(acc_cells))))
        out = A.Out()
        dropped = C.c_int64(0)
        rc = lib().fwa_fire_partials(self.h, _ptr(rows), n, m, cells, int(wm), A.PUSH_DEVICE_PTRS if device else 0,
                                     C.byref(out), C.byref(dropped))
        self._settled()
        _check(rc, self.h)
        if not device_output:
            return self._rows(out)
        res = {f: dev_view(getattr(out, f), out.n_rows, np.dtype("i8")) for f in ("key", "win_start", "win_end")}
        for j, name in enumerate(self.names):
            res["agg%d" % j] = dev_view(out.agg[j], out.n_rows, np.dtype(A.AGG_RESULT_DTYPE[name]))
        return res

    # -- checkpoint / restore (HeapSnapshotStrategy + SlicingWindowOperator watermark state) --
    def snapshot(self):
        """Return the handle's keyed window state + watermark as bytes (key-group-partitioned blob,
        format in include/flink_amd.h; parse with flink_amd.snapshot.parse)."""
        b = Blob()
        rc = lib().fwa_snapshot(self.h, C.byref(b))
        self._settled()
        _check(rc, self.h)
        try:
            return C.string_at(b.data, b.size) if b.size else b""
        finally:
            lib().fwa_blob_free(C.byref(b))

    def restore(self, blobs):
        """Restore a fresh handle from one or more snapshots (only this handle's key groups are read;
        watermark = min over the snapshots)."""
        if isinstance(blobs, (bytes, bytearray)):
            blobs = [blobs]
        bufs = [C.create_string_buffer(bytes(b), len(b)) for b in blobs]
        ptrs = (C.c_void_p * max(1, len(bufs)))(*[C.cast(b, C.c_void_p).value for b in bufs])
        sizes = (C.c_int64 * max(1, len(bufs)))(*[len(b) for b in blobs])
        rc = lib().fwa_restore(self.h, ptrs, sizes, len(bufs))
        self._settled()
        _check(rc, self.h)

    def snapshot_heap(self, keydict=None):
        """Keyed window state in Flink's heap-backend key-group byte layout (fwa_snapshot_heap): returns
        (body bytes, per-key-group section offsets, watermark). keydict: the flink_amd.keydict.KeyDictionary of an
        engine on dictionary ids (key rows written as its multi-column BinaryRowData rows)."""
        b = Blob()
        nkg = self.cfg.kg_end - self.cfg.kg_start + 1
        offs = np.zeros(nkg, np.int64)
        wm = C.c_int64(0)
        if keydict is not None:
            rc = lib().fwa_snapshot_heap_keys(self.h, keydict.h, C.byref(b), offs.ctypes.data_as(C.c_void_p), C.byref(wm))
        else:
            rc = lib().fwa_snapshot_heap(self.h, C.byref(b), offs.ctypes.data_as(C.c_void_p), C.byref(wm))
        self._settled()
        _check(rc, self.h)
        try:
            return (C.string_at(b.data, b.size) if b.size else b""), offs, wm.value
        finally:
            lib().fwa_blob_free(C.byref(b))

    def restore_heap(self, bodies, watermarks, keydict=None):
        bufs = [C.create_string_buffer(bytes(b), max(1, len(b))) for b in bodies]
        ptrs = (C.c_void_p * len(bufs))(*[C.cast(b, C.c_void_p).value for b in bufs])
        sizes = (C.c_int64 * len(bufs))(*[len(b) for b in bodies])
        wms = (C.c_int64 * len(bufs))(*[int(w) for w in watermarks])
        if keydict is not None:
            rc = lib().fwa_restore_heap_keys(self.h, keydict.h, ptrs, sizes, wms, len(bufs))
        else:
            rc = lib().fwa_restore_heap(self.h, ptrs, sizes, wms, len(bufs))
        self._settled()
        _check(rc, self.h)

    def flush(self):
        rc = lib().fwa_flush(self.h)
        self._settled()
        _check(rc, self.h)

    @property
    def record_lists(self):
        """True when the handle keeps TUMBLE window state as record lists (FWA_CFG_RECORD_LISTS, chosen or auto)."""
        c = A.Config()
        _check(lib().fwa_get_config(self.h, C.byref(c)), self.h)
        return bool(c.flags & A.CFG_RECORD_LISTS)

    def stats(self):
        st = A.Stats()
        rc = lib().fwa_get_stats(self.h, C.byref(st))
        self._settled()
        _check(rc, self.h)
        return st

    def late_records(self):
        """Indices (into the last push's batch) of the records it dropped as late (FWA_CFG_LATE_INDICES)."""
        p, n = C.c_void_p(), C.c_int64()
        rc = lib().fwa_late_records(self.h, C.byref(p), C.byref(n))
        self._settled()
        _check(rc, self.h)
        if n.value == 0:
            return np.zeros(0, np.int32)
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_int32)), shape=(n.value,)).copy()

    def reset_timers(self):
        rc = lib().fwa_reset_timers(self.h)
        self._settled()
        _check(rc, self.h)

    def close(self):
        if self.h:
            lib().fwa_destroy(self.h)
            self.h = C.c_void_p()
            self._inflight = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _host_to_np(p, n, dt):
    if n == 0 or not p:
        return np.zeros(0, dt)
    buf = (C.c_char * (n * dt.itemsize)).from_address(p)
    return np.frombuffer(buf, dtype=dt, count=n).copy()


class _CudaArray:
    def __init__(self, p, n, dt):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": dt.str, "data": (int(p), False),
                                         "version": 3}


def dev_view(p, n, dt):
    """Zero-copy torch view of engine-owned device memory."""
    import torch
    if n == 0 or not p:
        return torch.zeros(0, dtype=getattr(torch, {"i8": "int64", "f4": "float32", "f8": "float64", "u1": "uint8"}[dt.str[1:]]),
                           device="cuda")
    return torch.as_tensor(_CudaArray(p, n, dt), device="cuda")


def _dev_to_np(p, n, dt):
    if n == 0 or not p:
        return np.zeros(0, dt)
    return dev_view(p, n, dt).cpu().numpy().copy()


def key_groups(keys, max_parallelism=128, parallelism=1, key_kind=A.KEY_JAVA_LONG, key_hash=None, device=0):
    """KeyGroupRangeAssignment on the GPU: (key_group, operator_index) int32 arrays."""
    dev = _is_torch_cuda(keys)
    if dev:
        import torch
        n = keys.shape[0]
        kg = torch.empty(n, dtype=torch.int32, device=keys.device)
        op = torch.empty(n, dtype=torch.int32, device=keys.device)
    else:
        keys = np.ascontiguousarray(keys, np.int64)
        n = keys.shape[0]
        kg = np.empty(n, np.int32)
        op = np.empty(n, np.int32)
        if key_hash is not None:
            key_hash = np.ascontiguousarray(key_hash, np.int32)
    rc = lib().fwa_key_groups(_ptr(keys), _ptr(key_hash), n, key_kind, max_parallelism, parallelism,
                              _ptr(kg), _ptr(op), A.PUSH_DEVICE_PTRS if dev else 0, device)
    _check(rc, None, "fwa_key_groups")
    return kg, op


def route_rows(keys, cols, max_parallelism, parallelism, key_kind=A.KEY_JAVA_LONG, key_hash=None):
    """keyBy send side on the GPU (fwa_route_rows): torch CUDA columns -> (int64 [n, len(cols)] rows grouped by
    destination subtask, in arrival order within one; int64 [parallelism] row counts). Runs on torch's current
    stream."""
    import torch
    n = int(keys.shape[0])
    dev = keys.device
    out = torch.empty((n, len(cols)), dtype=torch.int64, device=dev)
    counts = torch.empty(parallelism, dtype=torch.int64, device=dev)
    ptrs = (C.c_void_p * len(cols))(*[c.data_ptr() for c in cols])
    nbytes = (C.c_int32 * len(cols))(*[c.element_size() for c in cols])
    stream = torch.cuda.current_stream(dev).cuda_stream
    rc = lib().fwa_route_rows(_ptr(keys), _ptr(key_hash), n, key_kind, max_parallelism, parallelism, ptrs, nbytes,
                              len(cols), _ptr(out), _ptr(counts), dev.index or 0, C.c_void_p(stream))
    _check(rc, None, "fwa_route_rows")
    return out, counts


def unpack_rows(rows):
    """Packed int64 rows [n, m] (torch CUDA) -> m contiguous int64 columns (fwa_unpack_rows, one kernel)."""
    import torch
    n, m = int(rows.shape[0]), int(rows.shape[1])
    cols = [torch.empty(n, dtype=torch.int64, device=rows.device) for _ in range(m)]
    ptrs = (C.c_void_p * m)(*[c.data_ptr() for c in cols])
    stream = torch.cuda.current_stream(rows.device).cuda_stream
    rc = lib().fwa_unpack_rows(_ptr(rows.contiguous()), n, m, ptrs, rows.device.index or 0, C.c_void_p(stream))
    _check(rc, None, "fwa_unpack_rows")
    return cols


def generate(params, n, keys=None, ts=None, v_i64=None, v_f32=None, v_f64=None, device=0, stream=None):
    """Fill torch CUDA tensors with the synthetic stream of SURVEY.md §8(d) (device generator)."""
    rc = lib().fwa_generate(C.byref(params), n, _ptr(keys), _ptr(ts), _ptr(v_i64), _ptr(v_f32),
                            _ptr(v_f64), device, stream)
    _check(rc, None, "fwa_generate")


def version():
    return lib().fwa_version().decode()
