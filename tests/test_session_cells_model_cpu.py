"""Lane-level model of the sessions cell-path walk (sess3_segment_kernel's chunk body, DESIGN.md §4 "Cell path"), checked
against the interval union that defines merged sessions (MergingWindowSet.addWindow / TimeWindow.intersects: touching
windows merge). The model mirrors the kernel's wave-wide steps on 64 lanes -- group heads and segmented min / max scans
per (kid, cell) group joined with the pending group, packing of the ended groups, the head chain against the key's
running max end, accumulators scanned once per element segmented by session, and the carries between chunks -- so a
change to the kernel's logic can be checked here on the CPU first. CPU-only (no GPU, no oracle library).
"""
import random

import pytest

# Lane-level simulation of the sess3 chunk body (single-level accumulator scans), one wave walking [0, h1).
L = 64
def msb(m): return m.bit_length() - 1
def ffs(m): return (m & -m).bit_length() - 1 if m else -1
def popc(m): return bin(m).count("1")
def ballot(b): return sum(1 << i for i in range(L) if b[i])
def seg_scan(x, gs, op):
    # inclusive segmented scan: lane i combines [gs[i], i]
    out = list(x)
    for i in range(L):
        acc = None
        for j in range(gs[i], i + 1):
            acc = x[j] if acc is None else op(acc, x[j])
        out[i] = acc
    return out
def walk(elems, gap):
    # elems: list of (kid, cell, start, end, acc) sorted by (kid, cell); acc = count
    h1 = len(elems)
    SENT = None
    out = []
    gopen = copen = False
    gkey = ck = None; gmin = gmax = 0; cmaxe = -2**63; cst = 0; gacc = 0; cacc = 0
    for base in range(0, h1, 64):
        q = [base + i for i in range(L)]
        v = [qq < h1 for qq in q]
        bk = [(elems[qq][0], elems[qq][1]) if v[i] else SENT for i, qq in enumerate(q)]
        st = [elems[qq][2] if v[i] else 2**63 for i, qq in enumerate(q)]
        en = [elems[qq][3] if v[i] else -2**63 for i, qq in enumerate(q)]
        x = [elems[qq][4] if v[i] else 0 for i, qq in enumerate(q)]
        more = base + 64 < h1
        cont0 = gopen and bk[0] == gkey
        gf = [v[i] and ((not cont0) if i == 0 else bk[i] != bk[i - 1]) for i in range(L)]
        GF = ballot(gf)
        below = [(2 << i) - 1 for i in range(L)]
        before = [(1 << i) - 1 for i in range(L)]
        gs = [msb(GF & below[i]) if GF & below[i] else 0 for i in range(L)]
        gm = [GF & below[i] for i in range(L)]
        st = seg_scan(st, gs, min); en = seg_scan(en, gs, max)
        for i in range(L):
            if gm[i] == 0 and cont0:
                st[i] = min(gmin, st[i]); en[i] = max(gmax, en[i])
        nk0 = (elems[base + 64][0], elems[base + 64][1]) if more else SENT
        gt = [v[i] and (q[i] + 1 == h1 or (bk[i + 1] != bk[i] if i < 63 else nk0 != bk[i])) for i in range(L)]
        lv = min(63, h1 - 1 - base)
        P = ballot(gt)
        pend = ((P >> lv) & 1) == 0
        np_ = popc(P)
        kk = [None] * L; gst = [0] * L; m = [-2**63] * L; cstart = [0] * L; head = [False] * L; ptail = [False] * L; H = 0
        if np_:
            idx = [i for i in range(L) if gt[i]]
            for r, i in enumerate(idx):
                kk[r] = bk[i][0]; gst[r] = st[i]
            gen = [en[i] for i in idx] + [-2**63] * (L - np_)
            range_end = base + lv + 1 == h1
            pv = [r < np_ for r in range(L)]
            kc = [pv[r] and ((not copen or kk[r] != ck) if r == 0 else kk[r] != kk[r - 1]) for r in range(L)]
            KM = ballot(kc)
            ks = [msb(KM & below[r]) if KM & below[r] else 0 for r in range(L)]
            m = seg_scan(gen, ks, max)
            for r in range(L):
                if (KM & below[r]) == 0 and copen and cmaxe > m[r]: m[r] = cmaxe
            mprev = [cmaxe] + m[:-1]
            head = [pv[r] and (kc[r] or gst[r] > mprev[r]) for r in range(L)]
            H = ballot(head)
            for r in range(L):
                hb = H & below[r]
                cs = msb(hb) if hb else 0
                cstart[r] = cst if hb == 0 else gst[cs]
            ptail = [pv[r] and (range_end if r == np_ - 1 else bool((H >> (r + 1)) & 1)) for r in range(L)]
        tl = []; ghead = []
        for i in range(L):
            Pge = P & ~before[i]
            t = ffs(Pge) if Pge else 64
            rk = popc(P & ((1 << t) - 1 if t < 64 else (1 << 64) - 1))
            tl.append(t); ghead.append(t < 64 and bool((H >> rk) & 1))
        SS = ballot([v[i] and gf[i] and (tl[i] == 64 or ghead[i]) for i in range(L)]) | 1
        ss = [msb(SS & below[i]) for i in range(L)]
        g0end = P != 0
        pre_c = copen and g0end and (H & 1) == 0
        pre_g = cont0
        xs = seg_scan(x, ss, lambda p, y: p + y)
        for i in range(L):
            if ss[i] == 0 and pre_g: xs[i] += gacc
            if ss[i] == 0 and pre_c: xs[i] += cacc
        x = xs
        emit_c = copen and np_ > 0 and (H & 1) != 0
        if emit_c: out.append((ck, cst, cmaxe, cacc))
        for i in range(L):
            if gt[i]:
                r = popc(P & before[i])
                if ptail[r]: out.append((bk[i][0], cstart[r], m[r], x[i]))
        if np_:
            tlast = msb(P)
            ck = kk[np_ - 1]; cmaxe = m[np_ - 1]; cst = cstart[np_ - 1]; cacc = x[tlast]; copen = True
        gopen = pend
        if pend:
            gkey = bk[lv]; gmin = st[lv]; gmax = en[lv]; gacc = x[lv]
    return out
def ref(elems):
    # sessions per kid: union of intersecting intervals (touching merges)
    by = {}
    for kid, cell, s, e, a in elems: by.setdefault(kid, []).append((s, e, a))
    out = []
    for kid, lst in by.items():
        lst.sort()
        cs, ce, ca = lst[0]
        for s, e, a in lst[1:]:
            if s <= ce: ce = max(ce, e); ca += a
            else: out.append((kid, cs, ce, ca)); cs, ce, ca = s, e, a
        out.append((kid, cs, ce, ca))
    return out


@pytest.mark.parametrize("seed", range(4))
def test_cell_walk_model_matches_interval_union(seed):
    random.seed(seed)
    for _ in range(150):
        gap = random.choice([3, 5, 10])
        elems = []
        for kid in range(random.randint(1, 4)):
            for _ in range(random.randint(1, 150)):
                t = random.randint(0, random.choice([20, 100, 400]))
                if random.random() < 0.05:      # an in-flight session: end past start + gap, its own count
                    s, e, a = t, t + gap + random.randint(0, 30), random.randint(1, 5)
                else:                           # a record: window [ts, ts + gap), COUNT 1
                    s, e, a = t, t + gap, 1
                elems.append((kid, s // gap, s, e, a))
        elems.sort(key=lambda z: (z[0], z[1]))  # the 32-bit (kid, cell) sort; order inside a cell arbitrary
        assert sorted(walk(elems, gap)) == sorted(ref(elems))
