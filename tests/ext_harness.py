"""ctypes driver for libfastlane_ext.so's mini DuckDB executor (tests only).

Mirrors how DuckDB runs `SELECT <proj> FROM fn(args) LIMIT n` against the
extension's table functions (see duckdb-fastlane_amd/extension/harness)."""
from __future__ import annotations

import ctypes as C
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
LIB = ROOT / "duckdb-fastlane_amd" / "libfastlane_ext.so"


class ExtError(RuntimeError):
    pass


class Ext:
    def __init__(self):
        lib = C.CDLL(str(LIB))
        lib.fls_ext_open.restype = C.c_void_p
        lib.fls_ext_close.argtypes = [C.c_void_p]
        lib.fls_ext_last_error.restype = C.c_char_p
        lib.fls_ext_has_function.argtypes = [C.c_void_p, C.c_char_p]
        lib.fls_ext_query.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_char_p), C.c_int, C.c_int,
                                      C.POINTER(C.c_int), C.c_int, C.c_int64, C.POINTER(C.c_void_p)]
        lib.fls_ext_result_rows.restype = C.c_int64
        lib.fls_ext_result_rows.argtypes = [C.c_void_p]
        lib.fls_ext_result_cols.argtypes = [C.c_void_p]
        for f in ("fls_ext_result_name", "fls_ext_result_type"):
            getattr(lib, f).restype = C.c_char_p
            getattr(lib, f).argtypes = [C.c_void_p, C.c_int]
        lib.fls_ext_result_value.restype = C.c_char_p
        lib.fls_ext_result_value.argtypes = [C.c_void_p, C.c_int64, C.c_int]
        lib.fls_ext_result_free.argtypes = [C.c_void_p]
        lib.fls_ext_scan_count.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.POINTER(C.c_int), C.c_int,
                                           C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
        self.lib = lib
        self.db = lib.fls_ext_open()
        if not self.db:
            raise ExtError(lib.fls_ext_last_error().decode())

    def has_function(self, name: str) -> bool:
        return bool(self.lib.fls_ext_has_function(self.db, name.encode()))

    def has_named_parameter(self, fn: str, name: str, type_id: int = 0) -> bool:
        f = self.lib.fls_ext_has_named_parameter
        f.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_int]
        return bool(f(self.db, fn.encode(), name.encode(), type_id))

    def copy_mode(self, fmt: str, preserve: bool, batch_index: bool, opts=None):
        """(execution mode 0/1/2 = REGULAR/PARALLEL/BATCH or -1, desired batch rows or -1)"""
        f = self.lib.fls_ext_copy_mode
        f.argtypes = [C.c_void_p, C.c_char_p, C.c_int, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), C.c_int,
                      C.POINTER(C.c_int64)]
        opts = opts or {}
        keys = (C.c_char_p * max(1, len(opts)))(*[k.encode() for k in opts])
        vals = (C.c_char_p * max(1, len(opts)))(*[str(v).encode() for v in opts.values()])
        rows = C.c_int64()
        mode = f(self.db, fmt.encode(), int(preserve), int(batch_index), keys, vals, len(opts), C.byref(rows))
        return mode, rows.value

    def scalar0(self, name: str):
        """SELECT name() for a zero-argument scalar function (None: not registered)"""
        f = self.lib.fls_ext_scalar0
        f.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_int]
        buf = C.create_string_buffer(256)
        n = f(self.db, name.encode(), buf, 256)
        return None if n < 0 else buf.value.decode()

    @staticmethod
    def _where(where):
        """where: [(table column, expr)], expr per fls_ext_harness.cpp (e.g.
        ">= 1994-01-01", "IN AIR|MAIL", "OR < 3|> 40", "ISNULL", "OPT = 5")."""
        where = where or []
        cols = (C.c_int * max(1, len(where)))(*[c for c, _ in where])
        exprs = (C.c_char_p * max(1, len(where)))(*[e.encode() for _, e in where])
        return cols, exprs, len(where)

    def query(self, fn, *args, as_list=False, raw=False, proj=None, limit=-1, threads=1, where=None):
        """Returns (names, types, rows) with rows as lists of str/None.
        fn=None resolves args[0] through the replacement scans.
        An int argument is passed as an INTEGER value (type errors).
        where: WHERE clauses the executor pushes into the scan as TableFilters."""
        a = (C.c_char_p * max(1, len(args)))(*[(b"\x01%d" % x) if isinstance(x, int) else str(x).encode()
                                               for x in args])
        p = (C.c_int * len(proj))(*proj) if proj else None
        out = C.c_void_p()
        mode = 2 if raw else int(as_list)
        wc, we, wn = self._where(where)
        self.lib.fls_ext_query_where.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_char_p), C.c_int, C.c_int,
                                                 C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_int),
                                                 C.POINTER(C.c_char_p), C.c_int, C.c_int64, C.c_int,
                                                 C.POINTER(C.c_void_p)]
        rc = self.lib.fls_ext_query_where(self.db, fn.encode() if fn else None, a, len(args), mode, p,
                                          len(proj) if proj else 0, wc, we, wn, limit, threads, C.byref(out))
        if rc != 0:
            raise ExtError(self.lib.fls_ext_last_error().decode())
        r = out.value
        try:
            nc = self.lib.fls_ext_result_cols(r)
            names = [self.lib.fls_ext_result_name(r, c).decode() for c in range(nc)]
            types = [self.lib.fls_ext_result_type(r, c).decode() for c in range(nc)]
            rows = []
            for i in range(self.lib.fls_ext_result_rows(r)):
                row = []
                for c in range(nc):
                    v = self.lib.fls_ext_result_value(r, i, c)
                    row.append(None if v is None else v.decode())
                rows.append(row)
            return names, types, rows
        finally:
            self.lib.fls_ext_result_free(r)

    def scan_count(self, fn, path, proj=None, threads=1, where=None):
        """(rows, checksum, seconds); the checksum depends only on the result
        rows in order (not on chunking or the number of scan threads)."""
        p = (C.c_int * len(proj))(*proj) if proj else None
        rows, h, sec = C.c_uint64(), C.c_uint64(), C.c_double()
        wc, we, wn = self._where(where)
        self.lib.fls_ext_scan_count_where.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.POINTER(C.c_int),
                                                      C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_char_p), C.c_int,
                                                      C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                                      C.POINTER(C.c_double)]
        rc = self.lib.fls_ext_scan_count_where(self.db, fn.encode(), str(path).encode(), p, len(proj) if proj else 0,
                                               wc, we, wn, threads, C.byref(rows), C.byref(h), C.byref(sec))
        if rc != 0:
            raise ExtError(self.lib.fls_ext_last_error().decode())
        return rows.value, h.value, sec.value

    def close(self):
        if self.db:
            self.lib.fls_ext_close(self.db)
            self.db = None

    def has_copy_function(self, name: str) -> bool:
        self.lib.fls_ext_has_copy_function.argtypes = [C.c_void_p, C.c_char_p]
        return bool(self.lib.fls_ext_has_copy_function(self.db, name.encode()))

    def copy(self, fn, src, dst, fmt="fls", proj=None, threads=1, **options):
        """COPY (SELECT <proj> FROM fn(src)) TO dst (FORMAT fmt, key value ...);
        returns the number of rows copied.  threads > 1: an unordered COPY with
        a parallel scan and a sink per thread (PARALLEL_COPY_TO_FILE)."""
        lib = self.lib
        lib.fls_ext_copy_mt.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.POINTER(C.c_int), C.c_int, C.c_char_p,
                                        C.c_char_p, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), C.c_int, C.c_int,
                                        C.POINTER(C.c_uint64)]
        keys = list(options)
        k = (C.c_char_p * max(1, len(keys)))(*[x.encode() for x in keys])
        v = (C.c_char_p * max(1, len(keys)))(*[str(options[x]).encode() for x in keys])
        p = (C.c_int * len(proj))(*proj) if proj else None
        rows = C.c_uint64()
        rc = lib.fls_ext_copy_mt(self.db, fn.encode(), str(src).encode(), p, len(proj) if proj else 0,
                                 fmt.encode(), str(dst).encode(), k, v, len(keys), threads, C.byref(rows))
        if rc != 0:
            raise ExtError(lib.fls_ext_last_error().decode())
        return rows.value

    def copy_values(self, columns, dst, fmt="fls", threads=1, **opts):
        """COPY (SELECT * FROM (VALUES ...)) TO dst (FORMAT fmt, opts): columns =
        [(name, "INTEGER" | "BIGINT" | "DOUBLE" | "VARCHAR", [values, None = NULL])].
        threads > 1: a parallel (unordered) COPY, chunk k sunk by thread k % threads."""
        lib = self.lib
        lib.fls_ext_copy_values_mt.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_int, C.POINTER(C.c_char_p),
                                               C.POINTER(C.c_char_p), C.c_int64, C.POINTER(C.c_char_p),
                                               C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), C.c_int, C.c_int,
                                               C.POINTER(C.c_uint64)]
        nc = len(columns)
        nr = len(columns[0][2]) if columns else 0
        names = (C.c_char_p * nc)(*[c[0].encode() for c in columns])
        types = (C.c_char_p * nc)(*[c[1].encode() for c in columns])
        cells = (C.c_char_p * max(1, nc * nr))()
        for r in range(nr):
            for j, c in enumerate(columns):
                v = c[2][r]
                cells[r * nc + j] = None if v is None else str(v).encode()
        keys = (C.c_char_p * max(1, len(opts)))(*[k.encode() for k in opts])
        vals = (C.c_char_p * max(1, len(opts)))(*[str(v).encode() for v in opts.values()])
        rows = C.c_uint64()
        rc = lib.fls_ext_copy_values_mt(self.db, fmt.encode(), str(dst).encode(), nc, names, types, nr, cells,
                                        keys, vals, len(opts), threads, C.byref(rows))
        if rc != 0:
            raise ExtError(lib.fls_ext_last_error().decode())
        return rows.value

    def scan_rows(self, fn, path, proj=None, threads=1):
        """DataChunk delivery only (a sink that counts rows): (rows, seconds)."""
        lib = self.lib
        lib.fls_ext_scan_rows.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.POINTER(C.c_int), C.c_int, C.c_int,
                                          C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
        p = (C.c_int * len(proj))(*proj) if proj else None
        rows, sec = C.c_uint64(), C.c_double()
        rc = lib.fls_ext_scan_rows(self.db, fn.encode(), str(path).encode(), p, len(proj) if proj else 0, threads,
                                   C.byref(rows), C.byref(sec))
        if rc != 0:
            raise ExtError(lib.fls_ext_last_error().decode())
        return rows.value, sec.value

    def facade_read(self, path, max_rows=-1, max_chunks=4096):
        """ext_fastlane::FastLanesFacade's read API (openFile, getColumnTypes,
        getColumnNames, readNextChunk(vector<Value>&, idx_t&)) as the
        reference's intended scanner drives it: (names, types, rows as lists of
        str/None, rows per readNextChunk call)."""
        lib = self.lib
        f = lib.fls_ext_facade_read
        f.argtypes = [C.c_char_p, C.c_int64, C.POINTER(C.c_void_p), C.POINTER(C.c_int64), C.c_int,
                      C.POINTER(C.c_int)]
        out = C.c_void_p()
        chunks = (C.c_int64 * max_chunks)()
        nch = C.c_int()
        if f(str(path).encode(), max_rows, C.byref(out), chunks, max_chunks, C.byref(nch)) != 0:
            raise ExtError(lib.fls_ext_last_error().decode())
        r = out.value
        try:
            nc = lib.fls_ext_result_cols(r)
            names = [lib.fls_ext_result_name(r, c).decode() for c in range(nc)]
            types = [lib.fls_ext_result_type(r, c).decode() for c in range(nc)]
            rows = []
            for i in range(lib.fls_ext_result_rows(r)):
                rows.append([None if (v := lib.fls_ext_result_value(r, i, c)) is None else v.decode()
                             for c in range(nc)])
            return names, types, rows, list(chunks[:min(nch.value, max_chunks)])
        finally:
            lib.fls_ext_result_free(r)

    def scan_hold(self, fn, path, threads=1):
        """Scan keeping a reference to every chunk until the end, then hash
        them (same checksum as scan_count): (rows, checksum, seconds)."""
        lib = self.lib
        lib.fls_ext_scan_hold.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_int, C.POINTER(C.c_uint64),
                                          C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
        rows, h, sec = C.c_uint64(), C.c_uint64(), C.c_double()
        rc = lib.fls_ext_scan_hold(self.db, fn.encode(), str(path).encode(), threads, C.byref(rows), C.byref(h),
                                   C.byref(sec))
        if rc != 0:
            raise ExtError(lib.fls_ext_last_error().decode())
        return rows.value, h.value, sec.value
