"""duckdb-fastlane_amd -- MI355X FastLanes scan path, Python binding.

Thin ctypes view of the C-ABI in include/flsgpu.h and include/flswriter.h
(libflsgpu.so, built in-tree by `make -C duckdb-fastlane_amd`).  It exists for
tests and bench.py; the product boundary is the C-ABI itself, consumed by the
C++ DuckDB glue in extension/.  There is no CPU fallback: if the shared library
is missing, importing this package raises.

Load with pkgload.load() (the directory name has a hyphen).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
# FLS_LIB selects an alternative in-tree build (A/B measurement of kernel variants)
LIB_PATH = _HERE / os.environ.get("FLS_LIB", "libflsgpu.so")

if not LIB_PATH.exists():
    raise ImportError(f"{LIB_PATH} not built: run `make -C {_HERE}` (hipcc --offload-arch=gfx950)")

_lib = C.CDLL(str(LIB_PATH))

# --- enums (include/flswriter.h) -------------------------------------------
INT8, INT16, INT32, INT64, UINT8, UINT16, UINT32, UINT64 = 1, 2, 3, 4, 5, 6, 7, 8
BOOLEAN, DATE, DECIMAL, FLOAT, DOUBLE, VARCHAR, BLOB = 9, 10, 11, 12, 13, 20, 21
STRING_TYPES = (VARCHAR, BLOB)
ENC_AUTO, ENC_FFOR, ENC_DELTA, ENC_DICT, ENC_RLE, ENC_ALP, ENC_FSST = 0, 1, 2, 3, 4, 5, 7

NP_DTYPE = {INT8: np.int8, INT16: np.int16, INT32: np.int32, INT64: np.int64,
            UINT8: np.uint8, UINT16: np.uint16, UINT32: np.uint32, UINT64: np.uint64,
            BOOLEAN: np.uint8, DATE: np.int32, DECIMAL: np.int64, FLOAT: np.float32, DOUBLE: np.float64}
TYPE_NAMES = {INT8: "TINYINT", INT16: "SMALLINT", INT32: "INTEGER", INT64: "BIGINT",
              UINT8: "UTINYINT", UINT16: "USMALLINT", UINT32: "UINTEGER", UINT64: "UBIGINT",
              DATE: "DATE", DECIMAL: "DECIMAL", FLOAT: "FLOAT", DOUBLE: "DOUBLE", VARCHAR: "VARCHAR",
              BOOLEAN: "BOOLEAN", BLOB: "BLOB"}
ROWGROUP = 65536


class FlsError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code
        self.msg = msg


class ColumnInfo(C.Structure):
    _fields_ = [("name", C.c_char_p), ("type", C.c_uint8), ("width", C.c_uint8),
                ("scale", C.c_uint8), ("out_bytes", C.c_uint8)]


class RowGroup(C.Structure):
    _fields_ = [("rowgroup", C.c_uint32), ("nrows", C.c_uint32), ("first_row", C.c_uint64),
                ("ncols", C.c_uint32), ("columns", C.POINTER(C.c_void_p)),
                ("nrows_scanned", C.c_uint32), ("sel", C.POINTER(C.c_uint32)),
                ("validity", C.POINTER(C.c_void_p)), ("dict", C.POINTER(C.c_void_p)),
                ("dict_size", C.POINTER(C.c_uint32)), ("dict_width", C.POINTER(C.c_uint8)),
                ("narrow", C.POINTER(C.c_uint8)), ("narrow_base", C.POINTER(C.c_uint64))]


class Predicate(C.Structure):
    _fields_ = [("col", C.c_uint32), ("clause", C.c_uint32), ("op", C.c_uint8), ("pad", C.c_uint8 * 7),
                ("value", C.c_uint64), ("str", C.c_char_p), ("str_len", C.c_uint64)]


# fls_cmp (include/flsgpu.h)
EQ, NE, LT, LE, GT, GE, IS_NULL, IS_NOT_NULL = range(8)
OPS = {"=": EQ, "==": EQ, "!=": NE, "<>": NE, "<": LT, "<=": LE, ">": GT, ">=": GE,
       "is_null": IS_NULL, "is_not_null": IS_NOT_NULL, "false": 8}


class DecodeStats(C.Structure):
    _fields_ = [("kernel_ms", C.c_double), ("values", C.c_uint64), ("packed_bytes", C.c_uint64),
                ("meta_bytes", C.c_uint64), ("out_bytes", C.c_uint64), ("launches", C.c_uint32),
                ("timed_launches", C.c_uint32), ("kernel_ms_total", C.c_double)]

    @property
    def algo_bytes(self) -> int:
        return int(self.packed_bytes + self.meta_bytes + self.out_bytes)


class PartInfo(C.Structure):
    _fields_ = [("device", C.c_int), ("rg_begin", C.c_uint32), ("rg_end", C.c_uint32), ("first_row", C.c_uint64),
                ("nrows", C.c_uint64)]


def _sig(name, res, *args):
    f = getattr(_lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


_P = C.c_void_p
_sig("fls_last_error", C.c_char_p)
_sig("fls_version", C.c_char_p)
_sig("fls_config_default", C.c_int, C.c_char_p, C.POINTER(C.c_int64))
_sig("fls_config_value", C.c_int, C.c_char_p, C.POINTER(C.c_int64))
_sig("fls_config_count", C.c_int)
_sig("fls_config_name", C.c_char_p, C.c_int)
_sig("fls_device_count", C.c_int)
_sig("fls_connect", C.c_int, C.POINTER(C.c_int), C.c_int, C.POINTER(_P))
_sig("fls_disconnect", None, _P)
_sig("fls_connection_trim", C.c_int, _P, C.c_uint64, C.POINTER(C.c_uint64))
_sig("fls_release_device_memory", C.c_int, C.c_int, C.POINTER(C.c_uint64))
_sig("fls_resident_info", C.c_int, C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32))
_sig("fls_read_fls", C.c_int, _P, C.c_char_p, C.POINTER(_P))
_sig("fls_read_fls_image", C.c_int, _P, _P, C.c_uint64, C.c_int, C.POINTER(_P))
_sig("fls_table_close", None, _P)
_sig("fls_table_ncols", C.c_uint32, _P)
_sig("fls_table_nrows", C.c_uint64, _P)
_sig("fls_table_row_offset", C.c_uint64, _P)
_sig("fls_table_nrowgroups", C.c_uint32, _P)
_sig("fls_table_rowgroup_rows", C.c_int64, _P, C.c_uint32)
_sig("fls_table_column", C.c_int, _P, C.c_uint32, C.POINTER(ColumnInfo))
_sig("fls_materialize", C.c_int, _P, C.c_uint32, C.POINTER(C.c_uint8), C.POINTER(RowGroup))
_sig("fls_scan_begin", C.c_int, _P, C.POINTER(C.c_uint8), C.c_uint32, C.c_uint32)
_sig("fls_scan_next", C.c_int, _P, C.POINTER(RowGroup))
_sig("fls_scan_acquire", C.c_int, _P, C.POINTER(RowGroup))
_sig("fls_scan_release", C.c_int, _P, C.c_uint32)
_sig("fls_scan_filter", C.c_int, _P, C.POINTER(Predicate), C.c_uint32)
_sig("fls_scan_pruned", C.c_int, _P)
_sig("fls_table_zonemap", C.c_int, _P, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
     C.POINTER(C.c_uint32))
_sig("fls_scan_dict_codes", C.c_int, _P, C.c_int)
_sig("fls_scan_narrow", C.c_int, _P, C.c_int)
_sig("fls_scan_defer_records", C.c_int, _P, C.c_int)
_sig("fls_scan_build_records", C.c_int, _P, C.POINTER(RowGroup))
_sig("fls_table_validity", C.c_int, _P, C.c_uint32, C.c_uint32, C.POINTER(C.POINTER(C.c_uint64)))
_sig("fls_rowgroup_may_match", C.c_int, _P, C.c_uint32, C.POINTER(Predicate), C.c_uint32)
_sig("fls_device_upload", C.c_int, _P, C.c_uint32, C.c_uint32)
_sig("fls_device_decode", C.c_int, _P, C.POINTER(C.c_uint8))
_sig("fls_device_sync", C.c_int, _P, C.POINTER(DecodeStats))
_sig("fls_device_column", C.c_int, _P, C.c_uint32, C.POINTER(_P), C.POINTER(C.c_uint64))
_sig("fls_device_copy_out", C.c_int, _P, C.c_uint32, C.c_uint64, C.c_uint64, _P)
_sig("fls_device_rows", C.c_uint64, _P)
_sig("fls_device_heap", C.c_int, _P, C.c_uint32, C.POINTER(_P), C.POINTER(_P), C.POINTER(C.c_uint64))
_sig("fls_device_parts", C.c_int, _P)
_sig("fls_device_part", C.c_int, _P, C.c_uint32, C.POINTER(PartInfo))
_sig("fls_device_part_column", C.c_int, _P, C.c_uint32, C.c_uint32, C.POINTER(_P), C.POINTER(C.c_uint64))
_sig("fls_device_part_heap", C.c_int, _P, C.c_uint32, C.c_uint32, C.POINTER(_P), C.POINTER(_P), C.POINTER(C.c_uint64))
_sig("fls_writer_new", _P, C.c_uint64)
_sig("fls_writer_free", None, _P)
_sig("fls_writer_add_column", C.c_int, _P, C.c_char_p, C.c_uint8, C.c_uint8, C.c_uint8, C.c_uint8)
_sig("fls_writer_add_rowgroup", C.c_int, _P, C.c_uint32, C.POINTER(_P), C.POINTER(_P))
_sig("fls_writer_set_threads", C.c_int, _P, C.c_int)
_sig("fls_writer_add_rowgroups", C.c_int, _P, C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(_P), C.POINTER(_P))
_sig("fls_writer_add_rowgroups_v", C.c_int, _P, C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(_P), C.POINTER(_P),
     C.POINTER(_P))
_sig("fls_writer_set_rowgroup_size", C.c_int, _P, C.c_uint32)
_sig("fls_writer_set_device", C.c_int, _P, C.c_int)
_sig("fls_device_alloc", C.c_int, C.c_int, C.c_uint64, C.POINTER(_P))
_sig("fls_device_free", C.c_int, C.c_int, _P)
_sig("fls_device_memcpy", C.c_int, C.c_int, _P, _P, C.c_uint64, C.c_int)
_sig("fls_encode_slot_bytes", C.c_uint64, C.c_uint8, C.c_uint8, C.c_uint32)
_sig("fls_encode_device", C.c_int, C.c_int, C.c_uint8, C.c_uint8, _P, C.c_uint64, C.c_uint32, _P,
     C.POINTER(C.c_uint64), C.POINTER(C.c_float))
_sig("fls_writer_finish_file", C.c_int, _P, C.c_char_p)
_sig("fls_writer_set_output", C.c_int, _P, C.c_char_p)
_sig("fls_writer_set_pipelined", C.c_int, _P, C.c_int)
_sig("fls_writer_finish_image", C.c_int, _P, C.POINTER(_P), C.POINTER(C.c_uint64))
_sig("fls_image_free", None, _P)
_sig("fls_gen_nrows", C.c_int64, C.c_char_p, C.c_double, C.c_uint64)
_sig("fls_gen_ncols", C.c_int, C.c_char_p)
_sig("fls_gen_image", C.c_int, C.c_char_p, C.c_double, C.c_uint64, C.c_uint32, C.c_uint32, C.c_int,
     C.POINTER(_P), C.POINTER(C.c_uint64))
_sig("fls_gen_values", C.c_int, C.c_char_p, C.c_double, C.c_uint64, C.c_int, C.c_uint64, C.c_uint64, _P)
_sig("fls_gen_dict_string", C.c_char_p, C.c_char_p, C.c_int, C.c_uint32)
_sig("fls_gen_strings", C.c_int64, C.c_char_p, C.c_double, C.c_uint64, C.c_int, C.c_uint64, C.c_uint64, _P, _P,
     C.c_uint64)

lib = _lib


def _check(rc: int) -> int:
    if rc < 0:
        raise FlsError(rc, (_lib.fls_last_error() or b"").decode(errors="replace"))
    return rc


def last_error() -> str:
    return (_lib.fls_last_error() or b"").decode(errors="replace")


def version() -> str:
    return _lib.fls_version().decode()


def config() -> dict[str, tuple[int, int]]:
    """The deployment knobs: name -> (compiled default, value in effect)."""
    out = {}
    for i in range(_lib.fls_config_count()):
        name = _lib.fls_config_name(i)
        d, v = C.c_int64(), C.c_int64()
        _check(_lib.fls_config_default(name, C.byref(d)))
        _check(_lib.fls_config_value(name, C.byref(v)))
        out[name.decode()] = (d.value, v.value)
    return out


def device_count() -> int:
    return _lib.fls_device_count()


# --- images ------------------------------------------------------------------
class Image:
    """An .fls file image in host memory (library-allocated, freed on close)."""

    def __init__(self, ptr: int, length: int):
        self.ptr, self.len = ptr, length

    def tobytes(self) -> bytes:
        return C.string_at(self.ptr, self.len)

    def view(self) -> np.ndarray:
        return np.ctypeslib.as_array(C.cast(self.ptr, C.POINTER(C.c_uint8)), shape=(self.len,))

    def write(self, path: str) -> None:
        Path(path).write_bytes(self.tobytes())

    def close(self) -> None:
        if self.ptr:
            _lib.fls_image_free(self.ptr)
            self.ptr = None

    def __del__(self):
        self.close()


def _take_image(rc, p, n) -> Image:
    _check(rc)
    return Image(p.value, n.value)


def gen_nrows(workload: str, scale: float = 1.0, nrows: int = 0) -> int:
    return _check(_lib.fls_gen_nrows(workload.encode(), scale, nrows))


def gen_image(workload: str, scale: float = 1.0, nrows: int = 0, rg_begin: int = 0,
              rg_end: int | None = None, nthreads: int | None = None) -> Image:
    if rg_end is None:
        rg_end = 0xFFFFFFFF
    if nthreads is None:
        nthreads = min(16, os.cpu_count() or 1)
    p, n = _P(), C.c_uint64()
    rc = _lib.fls_gen_image(workload.encode(), scale, nrows, rg_begin, rg_end, nthreads, C.byref(p), C.byref(n))
    return _take_image(rc, p, n)


def gen_values(workload: str, col: int, row_begin: int, n: int, dtype, scale: float = 1.0,
               nrows: int = 0) -> np.ndarray:
    out = np.empty(n, dtype=dtype)
    _check(_lib.fls_gen_values(workload.encode(), scale, nrows, col, row_begin, n, out.ctypes.data))
    return out


def gen_strings(workload: str, col: int, row_begin: int, n: int, scale: float = 1.0, nrows: int = 0) -> list[bytes]:
    """Ground-truth strings of a generated VARCHAR column (dictionary or l_comment)."""
    offs = np.zeros(n + 1, dtype=np.uint32)
    cap = max(64, 48 * n)
    buf = np.empty(cap, dtype=np.uint8)
    got = _lib.fls_gen_strings(workload.encode(), scale, nrows, col, row_begin, n, offs.ctypes.data, buf.ctypes.data,
                               cap)
    if got < 0:
        _check(int(got))
    b = buf[:got].tobytes()
    return [b[offs[i]:offs[i + 1]] for i in range(n)]


def gen_dict_string(workload: str, col: int, code: int) -> str | None:
    s = _lib.fls_gen_dict_string(workload.encode(), col, code)
    return None if s is None else s.decode()


# --- writer ----------------------------------------------------------------
def write_image(columns, rowgroup: int = ROWGROUP, row_offset: int = 0, device: int = -1,
                batch: int = 1, threads: int = 0, path: str | None = None, stream: bool = False,
                pipelined: bool = False) -> Image | None:
    """columns: list of (name, type, values, encoding[, width, scale]).
    values: numpy int array for integer types, float array for FLOAT/DOUBLE
    (stored bit-exactly), list of str/bytes for VARCHAR.  NULLs: None entries
    of a list, or the masked entries of a numpy.ma array (the rows' validity
    goes to fls_writer_add_rowgroups_v).  device >= 0: the
    FFOR / DELTA integer columns are encoded on that GPU (same bytes).
    batch > 1: row groups go in `batch` at a time (fls_writer_add_rowgroups;
    same bytes).  threads > 0: writer threads (fls_writer_set_threads).
    path: the file is written there instead (fls_writer_finish_file: the
    same bytes, chunks written in parallel, no image); returns None.
    stream: with path, row groups go to the file as they are encoded
    (fls_writer_set_output; the same bytes).  pipelined: a call returns
    before its row groups are encoded (fls_writer_set_pipelined; the same
    bytes), so each batch's buffers are kept until the next call returns."""
    w = _lib.fls_writer_new(row_offset)
    try:
        _check(_lib.fls_writer_set_rowgroup_size(w, rowgroup))
        if threads > 0:
            _check(_lib.fls_writer_set_threads(w, threads))
        if device >= 0:
            _check(_lib.fls_writer_set_device(w, device))
        if stream and path is not None:
            _check(_lib.fls_writer_set_output(w, str(path).encode()))
        if pipelined:
            _check(_lib.fls_writer_set_pipelined(w, 1))
        n = None
        held = None  # pipelined: the previous call's buffers
        prepped = []
        for spec in columns:
            name, ty, vals, enc = spec[:4]
            width, scale = (spec[4], spec[5]) if len(spec) > 4 else (0, 0)
            _check(_lib.fls_writer_add_column(w, name.encode(), ty, width, scale, enc))
            valid = None
            if isinstance(vals, np.ma.MaskedArray):
                valid = ~np.ma.getmaskarray(vals)
                vals = vals.filled(0)
            elif isinstance(vals, list) and any(v is None for v in vals):
                valid = np.array([v is not None for v in vals], dtype=bool)
                vals = [(b"" if ty in STRING_TYPES else 0) if v is None else v for v in vals]
            if ty in STRING_TYPES:
                bs = [v.encode() if isinstance(v, str) else bytes(v) for v in vals]
                prepped.append(("s", bs, valid))
                cnt = len(bs)
            else:
                arr = np.ascontiguousarray(np.asarray(vals).astype(NP_DTYPE[ty]))
                prepped.append(("i", arr, valid))
                cnt = len(arr)
            if n is None:
                n = cnt
            elif n != cnt:
                raise ValueError("columns differ in length")
        nc = len(prepped)
        starts = list(range(0, n or 0, rowgroup))
        for b0 in range(0, len(starts), max(1, batch)):
            grp = starts[b0:b0 + max(1, batch)]
            keep = []
            data = (_P * (nc * len(grp)))()
            offs = (_P * (nc * len(grp)))()
            vmask = (_P * (nc * len(grp)))()
            rows = (C.c_uint32 * len(grp))()
            for k, r0 in enumerate(grp):
                r1 = min(n, r0 + rowgroup)
                rows[k] = r1 - r0
                for c, (kind, v, valid) in enumerate(prepped):
                    if valid is not None:
                        words = np.packbits(valid[r0:r1], bitorder="little")
                        words = np.concatenate([words, np.zeros((-len(words)) % 8, np.uint8)]).view(np.uint64)
                        keep.append(words)
                        vmask[k * nc + c] = words.ctypes.data
                    if kind == "i":
                        part = np.ascontiguousarray(v[r0:r1])
                        keep.append(part)
                        data[k * nc + c] = part.ctypes.data
                    else:
                        sl = v[r0:r1]
                        o = np.zeros(len(sl) + 1, dtype=np.uint32)
                        o[1:] = np.cumsum([len(x) for x in sl], dtype=np.uint64).astype(np.uint32)
                        buf = np.frombuffer(b"".join(sl) or b"\0", dtype=np.uint8).copy()
                        keep += [o, buf]
                        data[k * nc + c] = buf.ctypes.data
                        offs[k * nc + c] = o.ctypes.data
            if any(p[2] is not None for p in prepped):
                _check(_lib.fls_writer_add_rowgroups_v(w, len(grp), rows, data, offs, vmask))
            elif batch > 1:
                _check(_lib.fls_writer_add_rowgroups(w, len(grp), rows, data, offs))
            else:
                _check(_lib.fls_writer_add_rowgroup(w, rows[0], data, offs))
            held = (keep, data, offs, vmask, rows)
        if path is not None:
            _check(_lib.fls_writer_finish_file(w, str(path).encode()))
            return None
        p, ln = _P(), C.c_uint64()
        rc = _lib.fls_writer_finish_image(w, C.byref(p), C.byref(ln))
        return _take_image(rc, p, ln)
    finally:
        _lib.fls_writer_free(w)


def encode_device(device: int, ty: int, enc: int, d_values: int, nrows: int, d_out: int,
                  rowgroup: int = ROWGROUP):
    """GPU chunk encoder over a device-resident column (fls_encode_device):
    d_values / d_out are device addresses (e.g. torch tensor data_ptr()).
    Returns (chunk lengths, kernel ms); chunk i starts at
    d_out + i * encode_slot_bytes(ty, enc, rowgroup)."""
    nrg = (nrows + rowgroup - 1) // rowgroup
    lens = (C.c_uint64 * nrg)()
    ms = C.c_float()
    _check(_lib.fls_encode_device(device, ty, enc, d_values, nrows, rowgroup, d_out, lens, C.byref(ms)))
    return [int(x) for x in lens], float(ms.value)


def encode_slot_bytes(ty: int, enc: int, rowgroup: int = ROWGROUP) -> int:
    return int(_lib.fls_encode_slot_bytes(ty, enc, rowgroup))


class DeviceBuffer:
    """A raw device allocation through the engine's own HIP runtime
    (fls_device_alloc): no second runtime (e.g. torch's) in the process."""

    def __init__(self, nbytes: int, device: int = 0):
        self.device, self.nbytes = device, int(nbytes)
        p = _P()
        _check(_lib.fls_device_alloc(device, self.nbytes, C.byref(p)))
        self.ptr = p.value

    @classmethod
    def from_array(cls, arr: np.ndarray, device: int = 0) -> "DeviceBuffer":
        arr = np.ascontiguousarray(arr)
        b = cls(arr.nbytes, device)
        _check(_lib.fls_device_memcpy(device, b.ptr, arr.ctypes.data, arr.nbytes, 0))
        return b

    def read(self, offset: int = 0, nbytes: int | None = None) -> bytes:
        n = self.nbytes - offset if nbytes is None else nbytes
        out = np.empty(n, dtype=np.uint8)
        if n:
            _check(_lib.fls_device_memcpy(self.device, out.ctypes.data, self.ptr + offset, n, 1))
        return out.tobytes()

    def free(self):
        if self.ptr:
            _lib.fls_device_free(self.device, self.ptr)
            self.ptr = None

    def __del__(self):
        self.free()


# --- engine ----------------------------------------------------------------
class Connection:
    """fastlanes::connect() counterpart: a set of GPUs to shard row groups over."""

    def __init__(self, devices=None):
        h = _P()
        if devices:
            arr = (C.c_int * len(devices))(*devices)
            _check(_lib.fls_connect(arr, len(devices), C.byref(h)))
        else:
            _check(_lib.fls_connect(None, 0, C.byref(h)))
        self.h = h.value
        self.devices = list(devices) if devices else [0]

    def trim(self, keep_bytes: int = 0) -> int:
        """Free idle scan pipelines down to keep_bytes of pinned memory per
        GPU; returns the pinned bytes still idle."""
        left = C.c_uint64()
        _check(_lib.fls_connection_trim(self.h, keep_bytes, C.byref(left)))
        return left.value

    @staticmethod
    def release_device_memory(device: int = -1) -> int:
        """Free the HBM-resident file images no running scan uses on device
        (-1: every GPU); returns the bytes freed (fls_release_device_memory)."""
        freed = C.c_uint64()
        _check(_lib.fls_release_device_memory(device, C.byref(freed)))
        return freed.value

    @staticmethod
    def resident_info(device: int = -1):
        """(bytes, images) of the HBM-resident file images on device (-1: all)."""
        b, n = C.c_uint64(), C.c_uint32()
        _check(_lib.fls_resident_info(device, C.byref(b), C.byref(n)))
        return b.value, n.value

    def read_fls(self, path: str) -> "Table":
        h = _P()
        _check(_lib.fls_read_fls(self.h, str(path).encode(), C.byref(h)))
        return Table(h.value, self)

    def read_image(self, img, copy: bool = False) -> "Table":
        h = _P()
        if hasattr(img, "ptr") and hasattr(img, "len"):  # an Image (possibly from another loaded build)
            _check(_lib.fls_read_fls_image(self.h, img.ptr, img.len, int(copy), C.byref(h)))
            t = Table(h.value, self)
            t._keep = img
            return t
        buf = bytes(img)
        _check(_lib.fls_read_fls_image(self.h, buf, len(buf), 1, C.byref(h)))
        return Table(h.value, self)

    def close(self):
        if self.h:
            _lib.fls_disconnect(self.h)
            self.h = None


def _mask(t: "Table", cols) -> C.Array | None:
    if cols is None:
        return None
    m = (C.c_uint8 * t.ncols)()
    for c in cols:
        m[c] = 1
    return m


class Table:
    def __init__(self, h, conn):
        self.h, self.conn, self._keep = h, conn, None

    def close(self):
        if self.h:
            _lib.fls_table_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def ncols(self) -> int:
        return _lib.fls_table_ncols(self.h)

    @property
    def nrows(self) -> int:
        return _lib.fls_table_nrows(self.h)

    @property
    def row_offset(self) -> int:
        return _lib.fls_table_row_offset(self.h)

    @property
    def nrowgroups(self) -> int:
        return _lib.fls_table_nrowgroups(self.h)

    def rowgroup_rows(self, rg: int) -> int:
        return _check(_lib.fls_table_rowgroup_rows(self.h, rg))

    def column(self, c: int) -> ColumnInfo:
        ci = ColumnInfo()
        _check(_lib.fls_table_column(self.h, c, C.byref(ci)))
        return ci

    def schema(self):
        out = []
        for c in range(self.ncols):
            ci = self.column(c)
            out.append((ci.name.decode(), ci.type, ci.width, ci.scale, ci.out_bytes))
        return out

    # -- host-delivered decode (DataChunk path)
    def _rg_arrays(self, rg: RowGroup, copy=True):
        cols = []
        sch = self.schema()
        for c in range(rg.ncols):
            p = rg.columns[c]
            if not p:
                cols.append(None)
                continue
            ob = sch[c][4]
            narrowed = bool(rg.narrow and rg.narrow[c])
            if (rg.dict and rg.dict[c]) or narrowed:
                ob = rg.dict_width[c]  # dictionary codes / narrowed values
            if rg.nrows == 0:
                cols.append(np.zeros(0, dtype=np.uint8))
                continue
            a = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(rg.nrows * ob,))
            if narrowed:  # widen: value = base + narrow (mod 2^64), in the column's width
                full = sch[c][4]
                w = a.view({1: np.uint8, 2: np.uint16, 4: np.uint32}[ob]).astype(np.uint64)
                v = (w + np.uint64(rg.narrow_base[c])).astype(np.uint64)
                a = v.view(np.uint8).reshape(-1, 8)[:, :full].reshape(-1).copy()
                cols.append(a)
                continue
            cols.append(a.copy() if copy else a)
        return cols

    @staticmethod
    def _rg_valid(rg: RowGroup):
        """per column: bool per delivered row (False = NULL), or None when every
        delivered row is valid (fls_rowgroup.validity)"""
        out = []
        for c in range(rg.ncols):
            p = rg.validity[c] if rg.validity else None
            if not p:
                out.append(None)
                continue
            nw = (rg.nrows + 63) // 64
            w = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint64)), shape=(max(1, nw),))
            out.append(np.unpackbits(w.view(np.uint8), bitorder="little")[:rg.nrows].astype(bool))
        return out

    def scan_nulls(self, cols=None, rg_begin=0, rg_end=None):
        """scan() that also yields each row group's validity and selection:
        (first_row, arrays, valid per column (None: no NULL), sel or None)"""
        if rg_end is None:
            rg_end = self.nrowgroups
        _check(_lib.fls_scan_begin(self.h, _mask(self, cols), rg_begin, rg_end))
        out = RowGroup()
        while _check(_lib.fls_scan_next(self.h, C.byref(out))) == 1:
            sel = np.ctypeslib.as_array(out.sel, shape=(out.nrows,)).copy() if out.sel and out.nrows else None
            yield out.first_row, self._rg_arrays(out), self._rg_valid(out), sel

    def narrow(self, enable: bool = True):
        """fls_scan_narrow: the next scan delivers integer columns narrowed to
        their row groups' ranges (scan() widens them back)"""
        _check(_lib.fls_scan_narrow(self.h, int(enable)))

    def dict_codes(self, enable: bool = True):
        """fls_scan_dict_codes: the next scan delivers DICT string columns as
        codes (scan_dicts yields their dictionaries)"""
        _check(_lib.fls_scan_dict_codes(self.h, int(enable)))

    def scan_dicts(self, cols=None, rg_begin=0, rg_end=None):
        """scan() yielding (first_row, arrays, dicts): dicts[c] is the row
        group's dictionary (string_t records, bytes) for a coded column, whose
        array then holds its codes (u8 / u16), else None"""
        if rg_end is None:
            rg_end = self.nrowgroups
        _check(_lib.fls_scan_begin(self.h, _mask(self, cols), rg_begin, rg_end))
        out = RowGroup()
        while _check(_lib.fls_scan_next(self.h, C.byref(out))) == 1:
            dicts = []
            for c in range(out.ncols):
                p = out.dict[c] if out.dict else None
                dicts.append(None if not p else np.ctypeslib.as_array(
                    C.cast(p, C.POINTER(C.c_uint8)), shape=(16 * out.dict_size[c],)).copy())
            arrays = self._rg_arrays(out)
            for c, dct in enumerate(dicts):
                if dct is not None:
                    arrays[c] = arrays[c].view(np.uint8 if out.dict_width[c] == 1 else np.uint16)
            yield out.first_row, arrays, dicts

    def validity(self, rg: int, col: int):
        """fls_table_validity: the chunk's validity words, or None (no NULL)"""
        p = C.POINTER(C.c_uint64)()
        if _check(_lib.fls_table_validity(self.h, rg, col, C.byref(p))) == 0:
            return None
        n = self.rowgroup_rows(rg)
        return np.ctypeslib.as_array(p, shape=(16 * ((n + 1023) // 1024),)).copy()

    def materialize(self, rg: int, cols=None):
        out = RowGroup()
        _check(_lib.fls_materialize(self.h, rg, _mask(self, cols), C.byref(out)))
        return out.first_row, self._rg_arrays(out)

    def scan(self, cols=None, rg_begin=0, rg_end=None):
        if rg_end is None:
            rg_end = self.nrowgroups
        _check(_lib.fls_scan_begin(self.h, _mask(self, cols), rg_begin, rg_end))
        out = RowGroup()
        while _check(_lib.fls_scan_next(self.h, C.byref(out))) == 1:
            yield out.first_row, self._rg_arrays(out)

    # -- pushed-down filters
    def _preds(self, filt):
        """filt: list of (col, op, value[, clause]); op a fls_cmp or one of OPS;
        value int (integers, DATE days, DECIMAL scaled), float (FLOAT/DOUBLE) or
        str/bytes (VARCHAR).  Terms without a clause get their own clause."""
        sch = self.schema()
        arr = (Predicate * max(1, len(filt)))()
        keep = []
        for i, term in enumerate(filt):
            col, op, val = term[:3]
            p = arr[i]
            p.col = col
            p.clause = term[3] if len(term) > 3 else 1000000 + i
            p.op = OPS[op] if isinstance(op, str) else op
            ty = sch[col][1] if 0 <= col < len(sch) else None
            if val is None or ty is None:
                pass
            elif ty in STRING_TYPES:
                b = val.encode() if isinstance(val, str) else bytes(val)
                buf = C.create_string_buffer(b, len(b) + 1)
                keep.append(buf)
                p.str = C.cast(buf, C.c_char_p)
                p.str_len = len(b)
            elif ty == FLOAT:
                p.value = int(np.array([val], dtype=np.float32).view(np.uint32)[0])
            elif ty == DOUBLE:
                p.value = int(np.array([val], dtype=np.float64).view(np.uint64)[0])
            else:
                p.value = int(val) & 0xFFFFFFFFFFFFFFFF
        return arr, len(filt), keep

    def set_filter(self, filt):
        arr, n, keep = self._preds(filt or [])
        _check(_lib.fls_scan_filter(self.h, arr, n))

    def may_match(self, rg: int, filt) -> bool:
        arr, n, keep = self._preds(filt)
        return _check(_lib.fls_rowgroup_may_match(self.h, rg, arr, n)) == 1

    @property
    def pruned(self) -> int:
        return _check(_lib.fls_scan_pruned(self.h))

    def zonemap(self, rg: int, col: int):
        """(min, max, flags) in the column's comparison domain, or None."""
        lo, hi, fl = C.c_uint64(), C.c_uint64(), C.c_uint32()
        if _check(_lib.fls_table_zonemap(self.h, rg, col, C.byref(lo), C.byref(hi), C.byref(fl))) == 0:
            return None
        ty = self.column(col).type
        if ty in (FLOAT, DOUBLE):
            cv = lambda x: float(np.array([x], dtype=np.uint64).view(np.float64)[0])  # noqa: E731
        elif ty in (INT8, INT16, INT32, INT64, DATE, DECIMAL):
            cv = lambda x: int(np.array([x], dtype=np.uint64).view(np.int64)[0])  # noqa: E731
        else:
            cv = int
        return cv(lo.value), cv(hi.value), fl.value

    def scan_filtered(self, filt, cols=None, rg_begin=0, rg_end=None):
        """Filtered scan: yields (rowgroup, first_row, sel, arrays) with only the
        qualifying rows (sel = their indices within the row group)."""
        if rg_end is None:
            rg_end = self.nrowgroups
        self.set_filter(filt)
        try:
            _check(_lib.fls_scan_begin(self.h, _mask(self, cols), rg_begin, rg_end))
            out = RowGroup()
            while _check(_lib.fls_scan_next(self.h, C.byref(out))) == 1:
                if out.sel:
                    sel = np.ctypeslib.as_array(out.sel, shape=(out.nrows,)).copy() if out.nrows else \
                        np.zeros(0, np.uint32)
                else:
                    sel = np.arange(out.nrows, dtype=np.uint32)
                yield out.rowgroup, out.first_row, sel, self._rg_arrays(out)
        finally:
            _check(_lib.fls_scan_filter(self.h, None, 0))

    # -- device-resident decode (bench)
    def device_upload(self, rg_begin=0, rg_end=None):
        if rg_end is None:
            rg_end = self.nrowgroups
        _check(_lib.fls_device_upload(self.h, rg_begin, rg_end))

    def device_decode(self, cols=None):
        _check(_lib.fls_device_decode(self.h, _mask(self, cols)))

    def device_sync(self) -> DecodeStats:
        st = DecodeStats()
        _check(_lib.fls_device_sync(self.h, C.byref(st)))
        return st

    def device_column(self, c: int):
        p, n = _P(), C.c_uint64()
        _check(_lib.fls_device_column(self.h, c, C.byref(p), C.byref(n)))
        return p.value, n.value

    def device_parts(self) -> list[PartInfo]:
        """The resident parts: one per GPU holding row groups (device_upload
        splits the range over the connection's GPUs)."""
        out = []
        for i in range(_lib.fls_device_parts(self.h)):
            pi = PartInfo()
            _check(_lib.fls_device_part(self.h, i, C.byref(pi)))
            out.append(pi)
        return out

    def device_part_column(self, part: int, c: int):
        p, n = _P(), C.c_uint64()
        _check(_lib.fls_device_part_column(self.h, part, c, C.byref(p), C.byref(n)))
        return p.value, n.value

    @property
    def device_rows(self) -> int:
        return _lib.fls_device_rows(self.h)

    def device_copy_out(self, c: int, row: int = 0, n: int | None = None) -> np.ndarray:
        ob = self.column(c).out_bytes
        if n is None:
            n = self.device_rows - row
        buf = np.empty(n * ob, dtype=np.uint8)
        _check(_lib.fls_device_copy_out(self.h, c, row, n, buf.ctypes.data))
        return buf


def as_values(raw: np.ndarray, ty: int) -> np.ndarray:
    """View decoded raw bytes of an integer column as its numpy dtype."""
    return raw.view(NP_DTYPE[ty])


def string_t_decode(raw: np.ndarray) -> list[bytes]:
    """Decode DuckDB string_t records (host pointers dereferenced for >12 B)."""
    rec = raw.reshape(-1, 16)
    lens = rec[:, :4].copy().view(np.uint32).ravel()
    out = []
    for i in range(len(lens)):
        n = int(lens[i])
        if n <= 12:
            out.append(bytes(rec[i, 4:4 + n]))
        else:
            ptr = int(rec[i, 8:16].copy().view(np.uint64)[0])
            out.append(C.string_at(ptr, n))
    return out


# --- full-size GPU verification (libflscheck.so; tests / bench support) ------
_check_lib = None


def _checklib():
    global _check_lib
    if _check_lib is None:
        path = _HERE / "libflscheck.so"
        if not path.exists():
            raise ImportError(f"{path} not built")
        lib_ = C.CDLL(str(path))
        lib_.fls_check_workload.restype = C.c_int
        lib_.fls_check_workload.argtypes = [C.c_char_p, C.c_double, C.c_uint64, C.c_uint64, C.c_uint64,
                                            C.POINTER(_P), C.POINTER(C.c_uint8), C.c_int, C.POINTER(_P),
                                            C.POINTER(C.c_int64), C.POINTER(C.c_uint64)]
        lib_.fls_check_workload_on.restype = C.c_int
        lib_.fls_check_workload_on.argtypes = [C.c_int] + lib_.fls_check_workload.argtypes
        lib_.fls_check_last_error.restype = C.c_char_p
        _check_lib = lib_
    return _check_lib


def check_device_table(t: "Table", workload: str, scale: float = 1.0, nrows: int = 0) -> list[int]:
    """Mismatching rows per column of t's resident decoded columns vs the
    workload generator (computed on the GPU holding each resident part).
    Call after device_sync()."""
    lib_ = _checklib()
    nc = t.ncols
    total = gen_nrows(workload, scale, nrows)
    obs = (C.c_uint8 * nc)(*[t.column(c).out_bytes for c in range(nc)])
    dicts = (_P * nc)()
    keep = []
    for c in range(nc):
        if obs[c] == 16:
            words = []
            k = 0
            while (s := gen_dict_string(workload, c, k)) is not None:
                words.append(s.encode())
                k += 1
            if words:
                b = C.create_string_buffer(b"\0".join(words) + b"\0\0")
                keep.append(b)
                dicts[c] = C.cast(b, _P)
    mism_total = [0] * nc
    for i, part in enumerate(t.device_parts()):
        cols = (_P * nc)()
        deltas = (C.c_int64 * nc)()
        for c in range(nc):
            cols[c] = t.device_part_column(i, c)[0]
            dp, hp, hn = _P(), _P(), C.c_uint64()
            if obs[c] == 16 and _lib.fls_device_part_heap(t.h, i, c, C.byref(dp), C.byref(hp), C.byref(hn)) == 1:
                deltas[c] = (dp.value or 0) - (hp.value or 0)   # free text (FSST): no dictionary
        mism = (C.c_uint64 * nc)()
        rc = lib_.fls_check_workload_on(part.device, workload.encode(), scale, total, t.row_offset + part.first_row,
                                        part.nrows, cols, obs, nc, dicts, deltas, mism)
        if rc != 0:
            raise FlsError(rc, lib_.fls_check_last_error().decode())
        mism_total = [a + b for a, b in zip(mism_total, mism)]
    return mism_total
