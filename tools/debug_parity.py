"""Diagnose a GPU-vs-oracle row mismatch of tests/test_gpu_parity.py::test_random_streams_vs_oracle (one config):
prints, per batch, the engine's adaptive modes and replay/straggler counters, and at the first mismatch the rows only
one side has (with their aggregates) plus both sides' rows of those keys. Usage: python tools/debug_parity.py CI AGGSET [OPTION=VALUE ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

from flink_amd import _abi as A  # noqa: E402
from flink_amd import engine  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402
import test_gpu_parity as T  # noqa: E402


def rows_of(r, names):
    out = []
    for i in range(len(r["key"])):
        out.append((int(r["key"][i]), int(r["win_start"][i]), int(r["win_end"][i])) +
                   tuple(r["agg%d" % j][i].item() for j in range(len(names))))
    return out


def mix64(x):
    """jm::mix64 (flink_amd/csrc/java_math.h): the key table's hash, to see where a key's probe starts."""
    M = (1 << 64) - 1
    z = x & M
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return z ^ (z >> 31)


def main():
    ci = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    aset = sys.argv[2] if len(sys.argv) > 2 else "i64"
    aggs = {"i64": T.I64_AGGS, "f64": T.F64_AGGS, "f32": T.F32_AGGS}[aset]
    opts = dict(a.split("=") for a in sys.argv[3:])      # e.g. window_passes=0 (fwa_set_option before the first push)
    engine.DEFAULT_OPTIONS.update({k: int(v) for k, v in opts.items()})
    cfg = A.make_config(aggs=aggs, key_capacity=4096, **T.CONFIGS[ci])
    names = A.agg_names(cfg)
    stream = T.random_stream(100 + ci, 40_000, 600, 60_000, 1500)
    g, o = engine.WindowAggregator(cfg), Oracle(cfg)
    for b, (k, t, cols, wm) in enumerate(T.batches_of(stream, 12, 1500)):
        dg, do = g.push(k, t, cols), o.push(k, t, cols)
        st = g.stats()
        modes = {m: g.get_option(m) for m in ("skew_merge", "window_passes", "narrow_entries")}
        print("batch %d n=%d wm=%d dropped %d/%d modes %s replay %d records_in %d live_slices %d" %
              (b, len(k), wm, dg, do, modes, st.replay_records, st.records_in, st.live_slices), flush=True)
        rg, ro = rows_of(g.advance_watermark(wm), names), rows_of(o.advance_watermark(wm), names)
        if sorted(rg) != sorted(ro):
            sg, so = sorted(rg), sorted(ro)
            only_g = [r for r in sg if r not in so]
            only_o = [r for r in so if r not in sg]
            print("MISMATCH at batch %d wm=%d: %d vs %d rows" % (b, wm, len(sg), len(so)))
            print("only GPU:", only_g[:20])
            print("only oracle:", only_o[:20])
            import collections
            dup = [kw for kw, c in collections.Counter(r[:3] for r in sg).items() if c > 1]
            print("(key, window) emitted more than once by the GPU:", len(dup))
            for kw in dup[:8]:
                print("  GPU:", [r for r in sg if r[:3] == kw], " ORA:", [r for r in so if r[:3] == kw],
                      " mix64 bucket:", hex(mix64(kw[0])))
            keys = sorted({r[0] for r in only_g + only_o} | {kw[0] for kw in dup})[:5]
            for kk in keys:
                print("key %d GPU:" % kk, [r for r in sg if r[0] == kk])
                print("key %d ORA:" % kk, [r for r in so if r[0] == kk])
                sel = k == kk
                print("key %d in this batch: ts %s" % (kk, sorted(t[sel].tolist())[:40]))
            return 1
    print("no mismatch")
    return 0


if __name__ == "__main__":
    sys.exit(main())
