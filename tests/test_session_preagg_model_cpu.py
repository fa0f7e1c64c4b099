"""Model of the sessions cell pre-aggregation path (flink_amd/csrc/sessions4.inc, DESIGN.md §5 "Cell pre-aggregation"),
checked against the interval union that defines merged sessions (MergingWindowSet.addWindow / TimeWindow.intersects:
windows [ts, ts + gap) that touch or overlap merge). The model follows the kernels' steps: cells of width gap aligned at
Long.MIN_VALUE (ord-encoded timestamp // gap), the cell's slot = cell % 16 with the walk starting at the push's first
cell, groups reduced to (count, min offset, max offset), a key's in-flight sessions sorted by start and merged with its
groups in start order, and the redo conditions (> 16 cells, > 8 sessions per key). CPU-only.
"""
import random

import pytest

CELLS, MAXS = 16, 8
M64 = (1 << 64) - 1


def ord64(x):
    return (x + (1 << 63)) & M64


def preagg(records, sessions, gap):
    """records: [(kid, ts)], sessions: {kid: [(start, end, count)]} -> ({kid: [(start, end, count)]}, redo)"""
    if not records:
        return None, True
    cells = [ord64(ts) // gap for _, ts in records]
    cmin, cmax = min(cells), max(cells)
    if cmax - cmin >= CELLS:
        return None, True
    base = cmin * gap                                     # ord-encoded first cell start
    table = {}
    for (kid, ts), c in zip(records, cells):
        slot = c % CELLS
        off = ord64(ts) - base
        assert 0 <= off < CELLS * gap
        g = table.setdefault((kid, slot), [0, 1 << 32, -1])
        g[0] += 1
        g[1] = min(g[1], off)
        g[2] = max(g[2], off)
    out = {}
    kids = {k for k, _ in records} | set(sessions)
    for kid in kids:
        ss = sorted(sessions.get(kid, []))
        if len(ss) > MAXS:
            return None, True
        items = []
        c0 = cmin % CELLS
        for j in range(CELLS):                            # cell order from the push's first cell
            g = table.get((kid, (c0 + j) % CELLS))
            if g:
                st = base + g[1] - (1 << 63)
                items.append(("g", st, base + g[2] - (1 << 63) + gap, g[0]))
        # merge by start: sessions first when starts tie (the kernel takes a session whose start <= the group's)
        merged, si = [], 0
        for it in items:
            while si < len(ss) and ss[si][0] <= it[1]:
                merged.append(("s",) + ss[si]); si += 1
            merged.append(it)
        merged += [("s",) + x for x in ss[si:]]
        res, cur = [], None
        for _, s, e, n in merged:
            if cur and s <= cur[1]:
                cur = [cur[0], max(cur[1], e), cur[2] + n]
            else:
                if cur:
                    res.append(tuple(cur))
                cur = [s, e, n]
        if cur:
            res.append(tuple(cur))
        out[kid] = res
    return out, False


def union(records, sessions, gap):
    out = {}
    kids = {k for k, _ in records} | set(sessions)
    for kid in kids:
        iv = [(ts, ts + gap, 1) for k, ts in records if k == kid] + list(sessions.get(kid, []))
        iv.sort()
        res = []
        for s, e, n in iv:
            if res and s <= res[-1][1]:
                ps, pe, pn = res[-1]
                res[-1] = (ps, max(pe, e), pn + n)
            else:
                res.append((s, e, n))
        out[kid] = res
    return out


@pytest.mark.parametrize("seed", range(200))
def test_preagg_model_matches_interval_union(seed):
    rng = random.Random(seed)
    gap = rng.choice([1, 7, 100, 1000, 5000])
    t0 = rng.choice([0, -10**12, 10**12, -2**62])
    span = rng.randint(1, 15 * gap)
    nk = rng.randint(1, 12)
    recs = [(rng.randrange(nk), t0 + rng.randrange(span)) for _ in range(rng.randint(1, 300))]
    if rng.random() < 0.3:                                # exact multiples of gap: touching windows
        recs += [(0, t0 + k * gap) for k in range(0, span // gap + 1)]
    sess = {}
    for kid in range(nk):
        if rng.random() < 0.5:
            s = t0 - rng.randint(0, 3 * gap)
            lst = []
            for _ in range(rng.randint(1, 3)):             # disjoint in-flight sessions (gaps of > 0)
                e = s + rng.randint(gap, 3 * gap)
                lst.append((s, e, rng.randint(1, 5)))
                s = e + rng.randint(1, 4 * gap)
            sess[kid] = lst
    got, redo = preagg(recs, sess, gap)
    if redo:                                               # > 16 cells: the sort-based path takes the push
        cells = [ord64(ts) // gap for _, ts in recs]
        assert max(cells) - min(cells) >= CELLS
        return
    exp = union(recs, sess, gap)
    assert {k: v for k, v in got.items() if v} == {k: v for k, v in exp.items() if v}


def test_cells_are_aligned_and_bounded():
    gap = 5000
    # a push of 75 s of event time (< 16 cells of 5 s) straddling a cell boundary anywhere stays on the path
    for t0 in (0, 4999, -1, -2**63 + 5, 2**62):
        recs = [(1, t0), (1, t0 + 74_999)]
        _, redo = preagg(recs, {}, gap)
        assert not redo
    _, redo = preagg([(1, 0), (1, 16 * gap)], {}, gap)
    assert redo
