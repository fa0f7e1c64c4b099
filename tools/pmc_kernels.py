"""Per-kernel average HBM bytes per dispatch from FETCH_SIZE / WRITE_SIZE passes (tools/gpu_pmc_c4_kernels.sh).

FETCH_SIZE is doubled (gfx950 correction, MI355X_MICROARCH.md); both counters are in KB.
Usage: python3 tools/pmc_kernels.py <dir with c4_FETCH_SIZE/ and c4_WRITE_SIZE/> [out.json]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import read  # noqa: E402


def main():
    d = sys.argv[1]
    fetch = read(os.path.join(d, "c4_FETCH_SIZE"))
    write = read(os.path.join(d, "c4_WRITE_SIZE"))
    out = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("sp_"):
            continue
        f = [v for _, v in fetch.get(k, [])][1:] or [v for _, v in fetch.get(k, [])]   # first dispatch is cold
        w = [v for _, v in write.get(k, [])][1:] or [v for _, v in write.get(k, [])]
        fb = 2 * 1024 * sum(f) / max(1, len(f))
        wb = 1024 * sum(w) / max(1, len(w))
        out[k] = {"read_bytes": fb, "write_bytes": wb, "dispatches": len(f)}
        print("%-20s read %8.3f GB  write %8.3f GB  per dispatch" % (k, fb / 1e9, wb / 1e9))
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
