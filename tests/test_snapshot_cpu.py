"""CPU tests: the snapshot blob reader against a blob laid out by hand per include/flink_amd.h."""
import numpy as np
import pytest

from flink_amd import snapshot as S


def make_blob(maxp=4, naggs=2, groups=((0, 2), (2, 1), (3, 3))):
    n = sum(c for _, c in groups)
    h = np.zeros(S.HDR_WORDS, "<i8")
    h[0] = np.int64(np.uint64(S.MAGIC).astype(np.int64))
    h[1] = 1
    h[2], h[4], h[9], h[11] = 0, 1000, maxp, naggs
    h[12], h[13] = 0, 1
    h[20], h[21], h[22], h[23] = 12345, n, 0, maxp - 1
    off = np.zeros(maxp + 1, "<i8")
    for g, c in groups:
        off[g + 1] = c
    off = np.cumsum(off)
    body = np.arange(n * (3 + naggs), dtype="<i8").reshape(3 + naggs, n)
    return np.concatenate([h, off, body.ravel()]).tobytes(), off, body


def test_parse_roundtrip():
    blob, off, body = make_blob()
    s = S.parse(blob)
    assert s["watermark"] == 12345 and s["n"] == 6 and s["max_parallelism"] == 4
    assert s["aggs"] == [0, 1]
    assert list(s["kg_offsets"]) == list(off)
    assert list(s["key"]) == list(body[0]) and list(s["acc"][1]) == list(body[4])
    assert s["key"][S.entries_of_key_group(s, 2)].tolist() == body[0][2:3].tolist()
    assert len(s["key"][S.entries_of_key_group(s, 1)]) == 0


def test_parse_rejects_bad_magic_and_size():
    blob, _, _ = make_blob()
    with pytest.raises(ValueError):
        S.parse(b"\0" + blob[1:])
    with pytest.raises(ValueError):
        S.parse(blob[:-8])
