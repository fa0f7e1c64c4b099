"""Key dictionary for multi-column Table keys (include/flink_amd.h fwa_keydict_*).

A Table job keyed by several fixed-length columns has BinaryRowData keys; KeyDictionary computes their
BinaryRowData.hashCode() (BinaryRowData.java:452-454, MurmurHashUtils.hashBytesByWords :92-170) on the GPU and maps
each distinct key row to an id carrying its key group (bits 48-63). An engine created with
key_kind=A.KEY_GROUP_PREFIXED aggregates on those ids; `decode` maps fired rows back to the key columns.
Columns are torch CUDA tensors (int64 BIGINT, int32 INT, float64 DOUBLE) or numpy arrays (copied to the device).
"""
import ctypes as C

import numpy as np

from .engine import EngineError, lib

FIELD = {"BIGINT": 0, "INT": 1, "DOUBLE": 2}
_DT = {0: np.int64, 1: np.int32, 2: np.float64}
_BOUND = False


def _bind():
    global _BOUND
    L = lib()
    if _BOUND:
        return L
    P = C.c_void_p
    L.fwa_keydict_create.argtypes = [C.c_int32, P, C.c_int32, C.c_int64, C.c_int32, C.POINTER(C.c_void_p)]
    L.fwa_keydict_create.restype = C.c_int
    L.fwa_keydict_destroy.argtypes = [P]
    L.fwa_keydict_destroy.restype = None
    L.fwa_keydict_last_error.argtypes = [P]
    L.fwa_keydict_last_error.restype = C.c_char_p
    L.fwa_keydict_size.argtypes = [P]
    L.fwa_keydict_size.restype = C.c_int64
    L.fwa_keydict_encode.argtypes = [P, P, P, C.c_int64, P, P]
    L.fwa_keydict_encode.restype = C.c_int
    L.fwa_keydict_decode.argtypes = [P, P, C.c_int64, P, P]
    L.fwa_keydict_decode.restype = C.c_int
    L.fwa_binrow_hash.argtypes = [C.c_int32, P, P, P, C.c_int64, P, C.c_int32]
    L.fwa_binrow_hash.restype = C.c_int
    _BOUND = True
    return L


def _dev(x, dtype):
    """A contiguous CUDA tensor of exactly `dtype`: the kernels read sizeof(dtype) bytes per row, so a narrower tensor
    would be read past its end and a host tensor would hand the GPU a host pointer."""
    import torch
    if type(x).__module__.startswith("torch"):
        if not x.is_cuda:
            raise TypeError("key columns must be CUDA tensors or numpy arrays (got a host tensor)")
        want = {np.dtype(np.int64): torch.int64, np.dtype(np.int32): torch.int32, np.dtype(np.float64): torch.float64,
                np.dtype(np.uint8): torch.uint8}[np.dtype(dtype)]
        if x.dtype != want and not (want == torch.uint8 and x.dtype == torch.bool):
            raise TypeError("key column of dtype %s where %s is expected" % (x.dtype, want))
        return x.contiguous().view(want) if x.dtype == torch.bool else x.contiguous()
    return torch.from_numpy(np.ascontiguousarray(x, dtype)).cuda()


def _ptrs(ts):
    return (C.c_void_p * max(1, len(ts)))(*[None if t is None else t.data_ptr() for t in ts])


def binrow_hash(types, cols, nulls=None, device=0):
    """BinaryRowData.hashCode() of each row of fixed-length fields (types: 'BIGINT' / 'INT' / 'DOUBLE')."""
    import torch
    L = _bind()
    tcodes = [FIELD[t] for t in types]
    dc = [_dev(c, _DT[k]) for c, k in zip(cols, tcodes)]
    dn = None if nulls is None else [None if z is None else _dev(z, np.uint8) for z in nulls]
    n = len(dc[0])
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    tarr = (C.c_int32 * len(tcodes))(*tcodes)
    rc = L.fwa_binrow_hash(len(tcodes), tarr, _ptrs(dc), None if dn is None else _ptrs(dn), n, out.data_ptr(), device)
    if rc:
        raise EngineError(rc, "fwa_binrow_hash")
    return out.cpu().numpy()


class KeyDictionary:
    def __init__(self, types, max_parallelism=128, capacity=1 << 20, device=0):
        L = _bind()
        self.types = [FIELD[t] for t in types]
        self.h = C.c_void_p()
        tarr = (C.c_int32 * len(self.types))(*self.types)
        rc = L.fwa_keydict_create(len(self.types), tarr, max_parallelism, capacity, device, C.byref(self.h))
        if rc:
            raise EngineError(rc, "fwa_keydict_create")

    def _check(self, rc, what):
        if rc:
            raise EngineError(rc, lib().fwa_keydict_last_error(self.h).decode() or what)

    def encode(self, cols, nulls=None, hashes=False):
        """ids (torch int64 CUDA tensor) of the key rows cols[c][i]; with hashes=True also their hashCode()."""
        import torch
        dc = [_dev(c, _DT[k]) for c, k in zip(cols, self.types)]
        dn = None if nulls is None else [None if z is None else _dev(z, np.uint8) for z in nulls]
        n = len(dc[0])
        ids = torch.empty(n, dtype=torch.int64, device="cuda")
        hs = torch.empty(n, dtype=torch.int32, device="cuda") if hashes else None
        torch.cuda.synchronize()
        self._check(lib().fwa_keydict_encode(self.h, _ptrs(dc), None if dn is None else _ptrs(dn), n, ids.data_ptr(),
                                              None if hs is None else hs.data_ptr()), "fwa_keydict_encode")
        return (ids, hs) if hashes else ids

    def decode(self, ids, with_nulls=True):
        """Key columns (numpy) and NULL flags of ids from this dictionary."""
        import torch
        di = _dev(ids, np.int64)
        n = len(di)
        cols = [torch.empty(n, dtype={0: torch.int64, 1: torch.int32, 2: torch.float64}[k], device="cuda")
                for k in self.types]
        nul = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in self.types] if with_nulls else None
        torch.cuda.synchronize()
        self._check(lib().fwa_keydict_decode(self.h, di.data_ptr(), n, _ptrs(cols), None if nul is None else _ptrs(nul)),
                    "fwa_keydict_decode")
        out = [c.cpu().numpy() for c in cols]
        return (out, [z.cpu().numpy().astype(bool) for z in nul]) if with_nulls else out

    def size(self):
        return int(lib().fwa_keydict_size(self.h))

    def close(self):
        if self.h:
            lib().fwa_keydict_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

