"""Key dictionary for multi-column Table keys (include/flink_amd.h fwa_keydict_*).

A Table job keyed by several fixed-length columns has BinaryRowData keys; KeyDictionary computes their
BinaryRowData.hashCode() (BinaryRowData.java:452-454, MurmurHashUtils.hashBytesByWords :92-170) on the GPU and maps
each distinct key row to an id carrying its key group (bits 48-63). An engine created with
key_kind=A.KEY_GROUP_PREFIXED aggregates on those ids; `decode` maps fired rows back to the key columns.
Columns are torch CUDA tensors of exactly the column's dtype (int64 BIGINT, int32 INT, float64 DOUBLE) or numpy
arrays (copied to the device); a host (CPU) torch tensor or a tensor of another dtype raises TypeError (the kernels
would read a host pointer or past the column's end), so callers holding CPU tensors pass `.numpy()` or `.cuda()`. A
STRING column is a sequence of str / bytes (UTF-8), or an (offsets int32 [n + 1], bytes uint8) pair of tensors.
"""
import ctypes as C

import numpy as np

from .engine import EngineError, lib

FIELD = {"BIGINT": 0, "INT": 1, "DOUBLE": 2, "STRING": 3}
STRING = 3


class KeyStrings(C.Structure):           # fwa_key_strings
    _fields_ = [("offsets", C.c_void_p), ("bytes", C.c_void_p)]


class KeyStringsOut(C.Structure):        # fwa_key_strings_out
    _fields_ = [("offsets", C.c_void_p), ("bytes", C.c_void_p), ("capacity", C.c_int64), ("needed", C.c_int64)]


def _str_col(x):
    """A STRING column -> (offsets int32 CUDA tensor [n + 1], bytes uint8 CUDA tensor)."""
    import torch
    if isinstance(x, tuple):
        return _dev(x[0], np.int32), _dev(x[1], np.uint8)
    bs = [b"" if v is None else (v.encode("utf-8") if isinstance(v, str) else bytes(v)) for v in x]
    offs = np.zeros(len(bs) + 1, np.int32)
    offs[1:] = np.cumsum([len(b) for b in bs], dtype=np.int64)
    data = np.frombuffer(b"".join(bs), np.uint8) if offs[-1] else np.zeros(1, np.uint8)
    return torch.from_numpy(offs).cuda(), torch.from_numpy(data.copy()).cuda()


def _cols_arg(types, cols):
    """The void* array fwa_keydict_encode / fwa_binrow_hash take, plus the objects it points into (kept alive)."""
    keep, ptrs = [], []
    for c, k in zip(cols, types):
        if k == STRING:
            o, b = _str_col(c)
            ks = KeyStrings(o.data_ptr(), b.data_ptr())
            keep += [o, b, ks]
            ptrs.append(C.addressof(ks))
        else:
            t = _dev(c, _DT[k])
            keep.append(t)
            ptrs.append(t.data_ptr())
    return (C.c_void_p * max(1, len(ptrs)))(*ptrs), keep
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
    carr, keep = _cols_arg(tcodes, cols)
    dn = None if nulls is None else [None if z is None else _dev(z, np.uint8) for z in nulls]
    n = len(cols[0]) if tcodes[0] != STRING or not isinstance(cols[0], tuple) else len(cols[0][0]) - 1
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    tarr = (C.c_int32 * len(tcodes))(*tcodes)
    torch.cuda.synchronize()
    rc = L.fwa_binrow_hash(len(tcodes), tarr, carr, None if dn is None else _ptrs(dn), n, out.data_ptr(), device)
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
        carr, keep = _cols_arg(self.types, cols)
        dn = None if nulls is None else [None if z is None else _dev(z, np.uint8) for z in nulls]
        c0 = cols[0]
        n = len(c0[0]) - 1 if isinstance(c0, tuple) else len(c0)
        ids = torch.empty(n, dtype=torch.int64, device="cuda")
        hs = torch.empty(n, dtype=torch.int32, device="cuda") if hashes else None
        torch.cuda.synchronize()
        self._check(lib().fwa_keydict_encode(self.h, carr, None if dn is None else _ptrs(dn), n, ids.data_ptr(),
                                              None if hs is None else hs.data_ptr()), "fwa_keydict_encode")
        return (ids, hs) if hashes else ids

    def decode(self, ids, with_nulls=True):
        """Key columns (numpy) and NULL flags of ids from this dictionary."""
        import torch
        di = _dev(ids, np.int64)
        n = len(di)
        cols, souts, ptrs = [], {}, []
        for c, k in enumerate(self.types):
            if k == STRING:                             # offsets first (bytes NULL: sizing), then the bytes
                o = torch.empty(n + 1, dtype=torch.int32, device="cuda")
                so = KeyStringsOut(o.data_ptr(), None, 0, 0)
                souts[c] = (o, so)
                cols.append(o)
                ptrs.append(C.addressof(so))
            else:
                t = torch.empty(n, dtype={0: torch.int64, 1: torch.int32, 2: torch.float64}[k], device="cuda")
                cols.append(t)
                ptrs.append(t.data_ptr())
        nul = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in self.types] if with_nulls else None
        carr = (C.c_void_p * max(1, len(ptrs)))(*ptrs)
        torch.cuda.synchronize()
        self._check(lib().fwa_keydict_decode(self.h, di.data_ptr(), n, carr, None if nul is None else _ptrs(nul)),
                    "fwa_keydict_decode")
        data = {}
        if souts:
            for c, (o, so) in souts.items():
                data[c] = torch.empty(max(1, so.needed), dtype=torch.uint8, device="cuda")
                so.bytes, so.capacity = data[c].data_ptr(), so.needed
            torch.cuda.synchronize()
            self._check(lib().fwa_keydict_decode(self.h, di.data_ptr(), n, carr, None if nul is None else _ptrs(nul)),
                        "fwa_keydict_decode")
        out = []
        for c, t in enumerate(cols):
            if c in souts:
                offs, raw = souts[c][0].cpu().numpy(), data[c].cpu().numpy().tobytes()
                out.append([raw[offs[i]:offs[i + 1]].decode("utf-8") for i in range(n)])
            else:
                out.append(t.cpu().numpy())
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

