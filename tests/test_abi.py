"""CPU tests: the C-ABI library exists, loads, and exports every symbol include/*.h declares."""
import ctypes
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "flink_amd", "libflink_amd.so")


def declared_symbols():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(fwa_\w+)\s*\(", src, flags=re.M):
            syms.add(m.group(1))
    return sorted(syms)


def test_header_declares_entry_points():
    s = declared_symbols()
    for need in ("fwa_create", "fwa_push", "fwa_advance_watermark", "fwa_flush", "fwa_destroy",
                 "fwa_last_error", "fwa_key_groups", "fwa_get_stats", "fwa_generate", "fwa_version"):
        assert need in s, need


def test_library_exports_every_declared_symbol():
    if not os.path.exists(LIB):
        pytest.fail("libflink_amd.so is not built; run __graft_entry__.build()")
    lib = ctypes.CDLL(LIB)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_version_string_without_gpu():
    lib = ctypes.CDLL(LIB)
    lib.fwa_version.restype = ctypes.c_char_p
    assert b"gfx950" in lib.fwa_version()


def test_struct_sizes_match_header():
    """ctypes mirror must match the C layout (compile a tiny probe with gcc)."""
    import subprocess
    import tempfile
    from flink_amd import _abi as A
    src = r'''
#include <stdio.h>
#include <stddef.h>
#include "flink_amd.h"
int main(void){printf("%zu %zu %zu %zu %zu\n", sizeof(fwa_config), sizeof(fwa_out), sizeof(fwa_stats),
 sizeof(fwa_gen_params), offsetof(fwa_config, aggs));return 0;}
'''
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "p.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "p")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        got = [int(x) for x in subprocess.check_output([exe]).split()]
    exp = [ctypes.sizeof(A.Config), ctypes.sizeof(A.Out), ctypes.sizeof(A.Stats), ctypes.sizeof(A.GenParams),
           A.Config.aggs.offset]
    assert got == exp


def test_stats_struct_size_pinned():
    """fwa_stats grew in ABI 5 (dec_inexact): the library reports its size and it equals the binding's."""
    from flink_amd import _abi as A
    from flink_amd import engine
    L = engine.lib()
    assert A.FWA_ABI_VERSION == 5
    assert L.fwa_stats_size() == ctypes.sizeof(A.Stats)


def test_engine_refuses_missing_library(tmp_path, monkeypatch):
    """The product path fails loudly (no CPU fallback) when the HIP library is absent."""
    from flink_amd import engine
    monkeypatch.setattr(engine, "_LIB", None)
    monkeypatch.setattr(engine, "LIB_PATH", str(tmp_path / "missing.so"))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        engine.lib()


def test_no_kernel_spills_vgprs():
    """Every gfx950 kernel of the library keeps its values in registers. A VGPR spill is not harmless with this
    toolchain: hipcc placed the spill stores of the combiner's prefetched entries before the exec-mask restore at a
    control-flow join, so lanes outside that branch lost their values (rel = 0 instead of -1 for padding lanes, whose
    key 0 was then counted in slice 0: the r04 window-pass parity failures, DESIGN.md section 4 "Skewed keys")."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from kernel_resources import kernels
    ks = kernels(LIB)
    assert len(ks) > 500
    spill = [(k["name"], k["vgpr_spill_count"]) for k in ks if k.get("vgpr_spill_count", 0) > 0]
    assert not spill, spill
