"""CPU tests of the multi-column key hash: the oracle's BinaryRowData.hashCode restatement
(oracle/fwa_oracle.c or_binrow_hash) against a second, byte-level restatement written here from the reference's
layout (BinaryRowData.java:68-123: 8-byte header with RowKind byte 0 and null bits from bit 8, one 8-byte slot per
fixed-length field) and hash (MurmurHashUtils.hashBytesByWords :92-170 over 4-byte little-endian words, seed 42,
fmix(h ^ length)). No reference test pins BinaryRowData hash values with literals: parity pinned by the
specification (two independent restatements) and, for one BIGINT field, by the single-field path the engine uses."""
import ctypes as C
import struct

import numpy as np
import pytest

from oracle import oracle as O

M32 = 0xFFFFFFFF


def _rotl(x, r):
    return ((x << r) | (x >> (32 - r))) & M32


def murmur_words(data, seed=42):
    """MurmurHashUtils.hashBytesByWords: mixK1 / mixH1 per 4-byte word, then fmix(h ^ length)."""
    h = seed
    for (w,) in struct.iter_unpack("<I", data):
        k = (w * 0xCC9E2D51) & M32
        k = _rotl(k, 15)
        k = (k * 0x1B873593) & M32
        h ^= k
        h = _rotl(h, 13)
        h = (h * 5 + 0xE6546B64) & M32
    h ^= len(data)
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 16
    return h - (1 << 32) if h >> 31 else h


def row_bytes(types, values):
    """BinaryRowData bytes of a row of fixed-length fields (None = NULL): header, then one slot per field."""
    hdr = 0
    slots = b""
    for i, (t, v) in enumerate(zip(types, values)):
        if v is None:
            hdr |= 1 << (i + 8)
            slots += b"\0" * 8
        elif t == "BIGINT":
            slots += struct.pack("<q", v)
        elif t == "INT":
            slots += struct.pack("<i", v) + b"\0" * 4
        else:
            slots += struct.pack("<d", v)
    return struct.pack("<Q", hdr) + slots


def oracle_hash(types, values):
    slots = np.zeros(len(types), np.int64)
    nb = 0
    for i, (t, v) in enumerate(zip(types, values)):
        if v is None:
            nb |= 1 << i
        elif t == "INT":
            slots[i] = v & M32
        elif t == "DOUBLE":
            slots[i] = struct.unpack("<q", struct.pack("<d", v))[0]
        else:
            slots[i] = v
    return O.lib().or_binrow_hash(slots.ctypes.data, len(types), nb)


def random_rows(rng, types, n, null_p):
    rows = []
    for _ in range(n):
        r = []
        for t in types:
            if rng.random() < null_p:
                r.append(None)
            elif t == "BIGINT":
                r.append(int(rng.integers(-2**63, 2**63 - 1)))
            elif t == "INT":
                r.append(int(rng.integers(-2**31, 2**31 - 1)))
            else:
                r.append(float(rng.choice([0.0, -0.0, 1.5, -3.25, rng.standard_normal() * 1e9, float("inf")])))
        rows.append(r)
    return rows


@pytest.mark.parametrize("types", [["BIGINT"], ["INT"], ["DOUBLE"], ["BIGINT", "INT"], ["INT", "DOUBLE", "BIGINT"],
                                   ["BIGINT"] * 4, ["INT", "INT", "DOUBLE", "BIGINT", "INT", "DOUBLE", "BIGINT", "INT"]])
def test_oracle_binrow_hash_matches_byte_restatement(types):
    rng = np.random.default_rng(len(types))
    for r in random_rows(rng, types, 300, 0.15):
        assert oracle_hash(types, r) == murmur_words(row_bytes(types, r)), r


def test_one_bigint_field_is_the_engine_single_key_hash():
    rng = np.random.default_rng(5)
    for v in [0, 1, -1, 2**63 - 1, -2**63] + [int(x) for x in rng.integers(-2**63, 2**63 - 1, 200)]:
        assert oracle_hash(["BIGINT"], [v]) == O.lib().or_binrow_bigint_hash(v)


def test_null_and_negative_zero_change_the_hash():
    """BinaryRowData equality is byte equality: NULL vs 0 and -0.0 vs 0.0 are different key rows."""
    assert oracle_hash(["BIGINT", "INT"], [None, 1]) != oracle_hash(["BIGINT", "INT"], [0, 1])
    assert oracle_hash(["DOUBLE"], [0.0]) != oracle_hash(["DOUBLE"], [-0.0])
    assert oracle_hash(["DOUBLE"], [0.0]) == murmur_words(row_bytes(["DOUBLE"], [0.0]))


def test_key_group_prefixed_ids():
    """FWA_KEY_GROUP_PREFIXED: the key group is the id's top 16 bits (a key dictionary's ids)."""
    for kg in (0, 5, 127):
        assert O.lib().or_key_group((kg << 48) | 12345, 3, 0, 128) == kg


def test_torch_key_columns_are_type_checked():
    """a torch key column must be a CUDA tensor of the field's exact dtype (the kernels read that many bytes
    per row); a host tensor is refused before anything reaches the GPU."""
    import torch
    from flink_amd import keydict
    with pytest.raises(TypeError):
        keydict._dev(torch.zeros(4, dtype=torch.int64), np.int64)
