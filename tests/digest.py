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


def row_hash(key, start, end, aggs):
    """or_row_digest of every row (int64 torch tensor, the uint64 value's bits)."""
    h = key * _s64(_K[0]) + start * _s64(_K[1]) + end * _s64(_K[2])
    for j, a in enumerate(aggs):
        h = h + a.to(torch.int64) * _s64(_K[3] + 2 * j)
    h = h ^ _lsr(h, 33)
    h = h * _s64(_K[4])
    h = h ^ _lsr(h, 29)
    h = h * _s64(_K[5])
    h = h ^ _lsr(h, 32)
    return h


def rows_digest(key, start, end, aggs):
    """(row count, digest as a Python int in [0, 2^64)) of int64 torch columns on any device."""
    return int(key.shape[0]), int(row_hash(key, start, end, aggs).sum().item()) % (1 << 64)


def f32_word(x):
    """A FLOAT result column as the oracle's 8-byte result word: the float's bits, zero-extended."""
    return x.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF


def f64_word(x):
    """A DOUBLE result column as the oracle's 8-byte result word: the double's bits."""
    return x.contiguous().view(torch.int64)


def bucket_sums(key, start, vals, nbuckets):
    """Per row bucket (or_row_digest(key, start, 0) & (nbuckets - 1)) the sums of each double column and of its
    magnitudes: float64 [len(vals), nbuckets] twice (or_pipeline_digests2's sum_mask side)."""
    b = row_hash(key, start, torch.zeros_like(key), []) & (nbuckets - 1)
    s = torch.zeros((len(vals), nbuckets), dtype=torch.float64, device=key.device)
    a = torch.zeros_like(s)
    for i, v in enumerate(vals):
        s[i].index_add_(0, b, v.to(torch.float64))
        a[i].index_add_(0, b, v.to(torch.float64).abs())
    return s, a
