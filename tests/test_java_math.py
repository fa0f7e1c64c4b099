"""CPU tests of the device math header compiled for the host with g++: magic division, Java '%',
window starts, murmur/key groups -- checked against the C oracle and Python big-int arithmetic."""
import ctypes
import os
import random
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROBE = r'''
#include <stdint.h>
#include "java_math.h"
extern "C" {
uint64_t t_udiv(uint64_t n, uint64_t d) { jm::UDiv64 v = jm::udiv64_make(d); return jm::udiv64(n, v); }
int64_t t_wstart(int64_t ts, int64_t off, int64_t size) { jm::UDiv64 v = jm::udiv64_make((uint64_t)size); return jm::window_start(ts, off, v); }
int32_t t_kg(int64_t key, int kind, int32_t h, int32_t maxp) { return jm::key_group(jm::key_hash(key, kind, h), maxp); }
int32_t t_murmur(int32_t c) { return jm::murmur_hash(c); }
}
'''


@pytest.fixture(scope="module")
def probe(tmp_path_factory):
    d = tmp_path_factory.mktemp("jm")
    src = d / "probe.cpp"
    src.write_text(PROBE)
    so = d / "probe.so"
    subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-I", os.path.join(ROOT, "flink_amd", "csrc"),
                           str(src), "-o", str(so)])
    L = ctypes.CDLL(str(so))
    L.t_udiv.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
    L.t_udiv.restype = ctypes.c_uint64
    L.t_wstart.argtypes = [ctypes.c_int64] * 3
    L.t_wstart.restype = ctypes.c_int64
    L.t_kg.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int32, ctypes.c_int32]
    L.t_kg.restype = ctypes.c_int32
    L.t_murmur.argtypes = [ctypes.c_int32]
    L.t_murmur.restype = ctypes.c_int32
    return L


def test_magic_division(probe):
    rng = random.Random(1)
    divisors = [1, 2, 3, 7, 10, 1000, 1024, 3600000, 10_000, 60_000, 86_400_000, 2**32 + 1, 2**63 - 1, 2**63,
                12345678901] + [rng.randrange(1, 2**64) for _ in range(200)]
    nums = [0, 1, 2**63 - 1, 2**63, 2**64 - 1] + [rng.randrange(0, 2**64) for _ in range(300)]
    for d in divisors:
        for n in nums:
            assert probe.t_udiv(n, d) == n // d, (n, d)


def test_window_start_matches_oracle(probe):
    rng = random.Random(2)
    L = O.lib()
    specials = [0, 1, -1, 4999, 5000, -5000, -4999, 2**63 - 1, -2**63, 2**63 - 1750]
    for size in [1, 7, 1000, 5000, 3600000, 86400000]:
        for off in [0, 100, -100, size - 1, -(size - 1)]:
            for ts in specials + [rng.randrange(-2**62, 2**62) for _ in range(200)]:
                assert probe.t_wstart(ts, off, size) == L.or_window_start(ts, off, size), (ts, off, size)


def test_key_groups_match_oracle(probe):
    rng = np.random.default_rng(3)
    L = O.lib()
    keys = np.concatenate([rng.integers(-2**63, 2**63 - 1, 2000, dtype=np.int64),
                           np.array([0, 1, -1, -2**63, 2**63 - 1], np.int64)])
    for kind in (0, 1, 2):
        for maxp in (128, 1, 7, 32768):
            for k in keys[:600]:
                h = int(k) & 0x7fffffff
                assert probe.t_kg(int(k), kind, h, maxp) == L.or_key_group(int(k), kind, h, maxp)
    for c in [0, 1, -1, 2**31 - 1, -2**31] + [int(x) for x in rng.integers(-2**31, 2**31 - 1, 500)]:
        assert probe.t_murmur(c) == L.or_murmur_hash(c)
