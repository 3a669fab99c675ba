"""ctypes wrapper of oracle/libflsref.so (CPU restatement, ORACLE).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the checker / timed CPU baseline.  PARITY
UNPINNED against upstream FastLanes bytes -- see flsref.h.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
LIB_PATH = _HERE / "libflsref.so"
if not LIB_PATH.exists():
    raise ImportError(f"{LIB_PATH} not built: run `make -C {_HERE}`")
_lib = C.CDLL(str(LIB_PATH))


class _File(C.Structure):
    _fields_ = [("img", C.c_void_p), ("len", C.c_size_t), ("ncols", C.c_uint32), ("nrows", C.c_uint64),
                ("nrowgroups", C.c_uint32), ("rowgroup_size", C.c_uint32), ("row_offset", C.c_uint64),
                ("footer", C.c_void_p), ("footer_len", C.c_uint32)]


_lib.flsref_tau.restype = C.c_uint32
_lib.flsref_tau.argtypes = [C.c_uint32]
_lib.flsref_unpack.restype = None
_lib.flsref_unpack.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p]
_lib.flsref_pack.restype = None
_lib.flsref_pack.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p]
_lib.flsref_open.restype = C.c_int
_lib.flsref_open.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(_File)]
_lib.flsref_column.restype = C.c_int
_lib.flsref_column.argtypes = [C.POINTER(_File), C.c_uint32, C.POINTER(C.c_int), C.POINTER(C.c_int),
                               C.POINTER(C.c_int), C.POINTER(C.c_char_p), C.POINTER(C.c_int)]
_lib.flsref_rowgroup_rows.restype = C.c_int64
_lib.flsref_rowgroup_rows.argtypes = [C.POINTER(_File), C.c_uint32]
_lib.flsref_decode.restype = C.c_int64
_lib.flsref_decode.argtypes = [C.POINTER(_File), C.c_uint32, C.c_uint32, C.c_void_p]
_lib.flsref_decode_column.restype = C.c_int64
_lib.flsref_decode_column.argtypes = [C.POINTER(_File), C.c_uint32, C.c_void_p, C.c_int]
_lib.flsref_decode_strings.restype = C.c_int64
_lib.flsref_decode_strings.argtypes = [C.POINTER(_File), C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64]
_lib.flsref_validity.restype = C.c_int
_lib.flsref_validity.argtypes = [C.POINTER(_File), C.c_uint32, C.c_uint32, C.c_void_p]
_lib.flsref_out_width.restype = C.c_int
_lib.flsref_out_width.argtypes = [C.POINTER(_File), C.c_uint32]


def tau(p: int) -> int:
    return _lib.flsref_tau(p)


def unpack(T: int, W: int, packed: bytes) -> np.ndarray:
    buf = np.frombuffer(bytes(packed) + b"\0" * 16, dtype=np.uint8)
    out = np.empty(1024, dtype=np.uint64)
    _lib.flsref_unpack(T, W, buf.ctypes.data, out.ctypes.data)
    return out


def pack(T: int, W: int, vals) -> bytes:
    v = np.ascontiguousarray(np.asarray(vals, dtype=np.uint64))
    out = np.zeros(128 * W + 16, dtype=np.uint8)
    _lib.flsref_pack(T, W, v.ctypes.data, out.ctypes.data)
    return out[:128 * W].tobytes()


class RefFile:
    """Oracle view of an .fls image (keeps the buffer alive)."""

    def __init__(self, img):
        if hasattr(img, "ptr") and hasattr(img, "len"):  # duckdb_fastlane_amd.Image
            self._keep = img
            ptr, n = img.ptr, img.len
        else:
            self._keep = np.frombuffer(bytes(img), dtype=np.uint8)
            ptr, n = self._keep.ctypes.data, len(self._keep)
        self.base = ptr
        self.f = _File()
        rc = _lib.flsref_open(ptr, n, C.byref(self.f))
        if rc != 0:
            raise ValueError(f"flsref_open failed: {rc}")

    @property
    def ncols(self):
        return self.f.ncols

    @property
    def nrows(self):
        return self.f.nrows

    @property
    def nrowgroups(self):
        return self.f.nrowgroups

    def column(self, c):
        t, w, s, nl = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        nm = C.c_char_p()
        assert _lib.flsref_column(C.byref(self.f), c, C.byref(t), C.byref(w), C.byref(s), C.byref(nm),
                                  C.byref(nl)) == 0
        return C.string_at(nm, nl.value).decode(), t.value, w.value, s.value

    def out_width(self, c) -> int:
        return _lib.flsref_out_width(C.byref(self.f), c)

    def rowgroup_rows(self, rg) -> int:
        return _lib.flsref_rowgroup_rows(C.byref(self.f), rg)

    def decode(self, c: int, rg: int) -> np.ndarray:
        """Raw decoded bytes of one chunk (ints: value width; VARCHAR: {u64 off, u64 len} pairs)."""
        n = self.rowgroup_rows(rg)
        out = np.empty(n * self.out_width(c), dtype=np.uint8)
        got = _lib.flsref_decode(C.byref(self.f), c, rg, out.ctypes.data)
        if got != n:
            raise ValueError(f"flsref_decode failed on col {c} rg {rg}")
        return out

    def decode_column(self, c: int, nthreads: int = 1) -> np.ndarray:
        out = np.empty(self.nrows * self.out_width(c), dtype=np.uint8)
        got = _lib.flsref_decode_column(C.byref(self.f), c, out.ctypes.data, nthreads)
        if got != self.nrows:
            raise ValueError(f"flsref_decode_column failed on col {c}")
        return out

    def strings_rg(self, c: int, rg: int) -> list[bytes]:
        """Strings of VARCHAR column c, row group rg (DICT or FSST)."""
        n = self.rowgroup_rows(rg)
        offs = np.zeros(n + 1, dtype=np.uint32)
        cap = 1 << 16
        while True:
            heap = np.empty(cap, dtype=np.uint8)
            got = _lib.flsref_decode_strings(C.byref(self.f), c, rg, offs.ctypes.data, heap.ctypes.data, cap)
            if got >= 0:
                break
            if cap > (1 << 34):
                raise ValueError(f"flsref_decode_strings failed on col {c} rg {rg}")
            cap *= 4
        hb = heap[:got].tobytes()
        return [hb[offs[i]:offs[i + 1]] for i in range(n)]

    def decode_strings_column(self, c: int, nthreads: int = 1) -> int:
        """Decode every row group of VARCHAR column c (DICT or FSST) into
        offsets + bytes, row groups spread over nthreads (ctypes releases the
        GIL); returns the string bytes produced.  CPU-baseline timing only."""
        from concurrent.futures import ThreadPoolExecutor

        def one(rg):
            n = self.rowgroup_rows(rg)
            offs = np.zeros(n + 1, dtype=np.uint32)
            cap = 64 * n + 4096
            while True:
                heap = np.empty(cap, dtype=np.uint8)
                got = _lib.flsref_decode_strings(C.byref(self.f), c, rg, offs.ctypes.data, heap.ctypes.data, cap)
                if got >= 0:
                    return got
                cap *= 4

        with ThreadPoolExecutor(max(1, nthreads)) as ex:
            return sum(ex.map(one, range(self.nrowgroups)))

    def validity(self, c: int, rg: int):
        """The chunk's validity words (u64, bit i of word j = row 64 j + i
        valid), or None when every row is valid (flsref_validity)."""
        n = self.rowgroup_rows(rg)
        words = np.zeros(16 * ((n + 1023) // 1024), dtype=np.uint64)
        got = _lib.flsref_validity(C.byref(self.f), c, rg, words.ctypes.data)
        if got < 0:
            raise ValueError(f"flsref_validity failed on col {c} rg {rg}")
        return words if got == 1 else None

    def valid_column(self, c: int) -> np.ndarray:
        """bool per row of column c: True where the row is not NULL"""
        parts = []
        for rg in range(self.nrowgroups):
            n = self.rowgroup_rows(rg)
            w = self.validity(c, rg)
            parts.append(np.ones(n, dtype=bool) if w is None
                         else np.unpackbits(w.view(np.uint8), bitorder="little")[:n].astype(bool))
        return np.concatenate(parts) if parts else np.zeros(0, dtype=bool)

    def strings_column(self, c: int) -> list[bytes]:
        out = []
        for rg in range(self.nrowgroups):
            out += self.strings_rg(c, rg)
        return out

    def strings(self, raw: np.ndarray) -> list[bytes]:
        pairs = raw.view(np.uint64).reshape(-1, 2)
        return [C.string_at(self.base + int(o), int(n)) for o, n in pairs]
