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


# ---- STRING fields (FWA_KEY_FIELD_STRING) ----------------------------------------------------------------------------

def test_fixed_part_sizes_match_the_reference():
    """BinaryRowDataTest.testBasic :92-95: fixed-length part sizes of arity 0 / 1 / 65 / 128 rows."""
    for arity, size in [(0, 8), (1, 16), (65, 536), (128, 1048)]:
        assert len(O.binrow_bytes(["BIGINT"] * arity, [0] * arity)) == size


def test_string_field_layout():
    """AbstractBinaryWriter.writeString: <= 7 bytes inline (0x80 | len in the top byte, bytes from the lowest), longer in
    the variable-length part, 8-byte aligned, slot = offset << 32 | length; the testWriter row (:131-148) shapes."""
    b = O.binrow_bytes(["STRING"], ["1234567"])
    assert len(b) == 16 and b[8:15] == b"1234567" and b[15] == 0x87
    b = O.binrow_bytes(["STRING"], ["12345678"])
    assert len(b) == 24 and struct.unpack("<Q", b[8:16])[0] == (16 << 32) | 8 and b[16:] == b"12345678"
    s = "啦啦啦啦啦我是快乐的粉刷匠".encode("utf-8")                       # 39 bytes -> 40 in the var part
    b = O.binrow_bytes(["STRING", "INT", "STRING"], ["1", 88, s])
    assert len(b) == 8 + 24 + 40 and struct.unpack("<Q", b[24:32])[0] == (32 << 32) | 39 and b[32:71] == s
    assert O.binrow_bytes(["STRING"], [""])[15] == 0x80 and O.binrow_bytes(["STRING"], [None])[8:] == bytes(8)
    assert b[1] == 0 and O.binrow_bytes(["INT", "STRING"], [1, None])[1] == 0b10


def test_bytes_hash_equals_the_fixed_row_hash():
    """The byte-level hash of a fixed-length row equals the oracle's slot-level BinaryRowData hash (and, for one
    BIGINT field, the single-key hash the engine uses), so the STRING rows share one hash definition with them."""
    rng = np.random.default_rng(9)
    for types in (["BIGINT"], ["INT", "DOUBLE", "BIGINT"]):
        for r in random_rows(rng, types, 100, 0.15):
            rb = O.binrow_bytes(types, r)
            assert O.binrow_hash_bytes(rb) == oracle_hash(types, r) == murmur_words(rb)
    for v in [0, -1, 2**63 - 1]:
        assert O.binrow_hash_bytes(O.binrow_bytes(["BIGINT"], [v])) == O.lib().or_binrow_bigint_hash(v)
    for s in ["", "a", "abcdefg", "abcdefgh", "啦啦啦啦啦我是快乐的粉刷匠" * 3]:
        rb = O.binrow_bytes(["STRING", "BIGINT"], [s, 7])
        assert O.binrow_hash_bytes(rb) == murmur_words(rb)


def test_string_hash_distribution_on_the_oracle():
    """BinaryRowDataTest :378-386 (scaled to 20,000 rows for the CPU suite; the GPU test runs the full 999,999)."""
    n = 20_000
    hs = {O.binrow_hash_bytes(O.binrow_bytes(["STRING"], ["啦啦啦啦啦我是快乐的粉刷匠%d" % i])) for i in range(n)}
    assert len(hs) > int(n * 0.997)
