"""Reader for fwa_snapshot blobs (layout in include/flink_amd.h, "checkpoint / restore").

The blob mirrors Flink's key-group-partitioned keyed-state snapshot: HeapSnapshotStrategy writes
each key group's state entries and a KeyGroupRangeOffsets index
(flink-runtime/.../state/heap/HeapSnapshotStrategy.java:154-179), so a restoring subtask reads only
the key groups it owns (StateAssignmentOperation). The operator's watermark travels with it, as
SlicingWindowOperator keeps it in union list state (SlicingWindowOperator.java:186-209).
"""
import numpy as np

MAGIC = 0x3150414E53415746   # "FWASNAP1" little-endian
HDR_WORDS = 32


def parse(blob):
    """Decode a snapshot into a dict: config fields, watermark, key-group offsets, SoA entry columns."""
    w = np.frombuffer(bytes(blob), dtype="<i8")
    if w.size < HDR_WORDS or int(w[0]) & 0xFFFFFFFFFFFFFFFF != MAGIC or int(w[1]) != 1:
        raise ValueError("not a flink_amd snapshot")
    maxp, naggs, n, nh = int(w[9]), int(w[11]), int(w[21]), int(w[25])
    session = int(w[2]) == 3                     # SESSION: a 4th leading column holds the session end (last)
    prehashed = int(w[10]) == 2                  # FWA_KEY_PREHASHED: a last column holds each key's key.hashCode()
    ncols = (4 if session else 3) + naggs + nh + (1 if prehashed else 0)   # nh: hidden non-NULL counters
    need = HDR_WORDS + maxp + 1 + n * ncols
    if w.size != need:
        raise ValueError("snapshot size %d words != %d" % (w.size, need))
    off = w[HDR_WORDS:HDR_WORDS + maxp + 1]
    body = w[HDR_WORDS + maxp + 1:].reshape(ncols, n) if n else np.zeros((ncols, 0), np.int64)
    out = {
        "window_kind": int(w[2]), "semantics": int(w[3]), "size_ms": int(w[4]), "slide_ms": int(w[5]),
        "offset_ms": int(w[6]), "gap_ms": int(w[7]), "allowed_lateness_ms": int(w[8]),
        "max_parallelism": maxp, "key_kind": int(w[10]), "aggs": [int(x) for x in w[12:12 + naggs]],
        "watermark": int(w[20]), "n": n, "kg_range": (int(w[22]), int(w[23])),
        "kg_offsets": off.copy(), "key": body[0].copy(), "slice_start": body[1].copy(),
        "count": body[2].copy(), "acc": [body[3 + j].copy() for j in range(naggs)],
        "nullable_cols": int(w[24]), "hidden": [body[3 + naggs + h].copy() for h in range(nh)],
    }
    if session:
        out["window_end"] = body[3 + naggs + nh].copy()   # slice_start holds the session start
    if prehashed:
        out["key_hash"] = body[ncols - 1].astype(np.int32)
    return out


def entries_of_key_group(snap, kg):
    """Slice of the entry columns belonging to key group kg (the KeyGroupRangeOffsets lookup)."""
    lo, hi = int(snap["kg_offsets"][kg]), int(snap["kg_offsets"][kg + 1])
    return slice(lo, hi)
