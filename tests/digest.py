"""TEST INFRASTRUCTURE: order-free digest of fired rows, computed with torch on the engine's device output columns.

Restates `or_row_digest` (oracle/fwa_oracle.c) in wrap-around int64 arithmetic: a linear mix of (key, window start,
window end, int64 aggregates) with odd constants, a 64-bit finalizer, summed mod 2^64 over a watermark's rows. Equal
digests and row counts per watermark mean equal row multisets up to a 2^-64 collision chance, whatever the emission
order (unspecified in the reference: TimerHeapInternalTimer.comparePriorityTo)."""
import torch

_K = (0x9E3779B97F4A7C15, 0xC2B2AE3D27D4EB4F, 0x165667B19E3779F9, 0xD6E8FEB86659FD93,
      0xC4CEB9FE1A85EC53, 0x94D049BB133111EB)


def _s64(c):
    return c - (1 << 64) if c >= 1 << 63 else c


def _lsr(x, s):
    return (x >> s) & ((1 << (64 - s)) - 1)


def rows_digest(key, start, end, aggs):
    """(row count, digest as a Python int in [0, 2^64)) of int64 torch columns on any device."""
    h = key * _s64(_K[0]) + start * _s64(_K[1]) + end * _s64(_K[2])
    for j, a in enumerate(aggs):
        h = h + a.to(torch.int64) * _s64(_K[3] + 2 * j)
    h = h ^ _lsr(h, 33)
    h = h * _s64(_K[4])
    h = h ^ _lsr(h, 29)
    h = h * _s64(_K[5])
    h = h ^ _lsr(h, 32)
    return int(key.shape[0]), int(h.sum().item()) % (1 << 64)
