"""NULLs: validity bitmaps in the container (csrc/fls_format.hpp "Validity").

The reference emits NULL for empty and unhandled columns
(/root/reference/src/fastlanes_facade.cpp:113-117,173-181) and its writer
tracks NULL strings (/root/reference/src/writer/write_fastlane.cpp:207-208);
here a column chunk with a NULL row stores nvec x 128 B of bitmaps (DuckDB's
ValidityMask layout) after its encoded values, whose NULL rows hold
placeholders.  CPU tests: the writer against the oracle (oracle/flsref.c
flsref_validity checks the bitmaps' bounds, padding and the vectors' has-NULL
marks); GPU tests: the C-ABI scan and read_fastlanes / COPY round trips."""
import numpy as np
import pytest

from ext_harness import Ext


@pytest.fixture(scope="module")
def ext(_built):
    e = Ext()
    yield e
    e.close()


def _null_mask(n, rng, p):
    v = rng.random(n) >= p
    return v


def _nullable_table(fl, n, seed, rowgroup=65536):
    """(image, cols, valid per column): every encoding with NULLs in varied
    densities, an all-NULL and a no-NULL column."""
    rng = np.random.default_rng(seed)
    valid = {
        "i32": _null_mask(n, rng, 0.1),
        "i64_delta": _null_mask(n, rng, 0.01),
        "u16_rle": _null_mask(n, rng, 0.5),
        "i8_dict": _null_mask(n, rng, 0.2),
        "dbl": _null_mask(n, rng, 0.05),
        "s_dict": _null_mask(n, rng, 0.3),
        "s_fsst": _null_mask(n, rng, 0.15),
        "all_null": np.zeros(n, dtype=bool),
        "no_null": np.ones(n, dtype=bool),
        "b": _null_mask(n, rng, 0.4),
    }
    if n > 3000:
        valid["i32"][1024:2048] = False           # a whole NULL vector
        valid["i32"][:5] = False                  # leading NULLs
    base = {
        "i32": (fl.INT32, rng.integers(-1000, 1000, n).astype(np.int32), fl.ENC_FFOR),
        "i64_delta": (fl.INT64, np.cumsum(rng.integers(0, 9, n)).astype(np.int64), fl.ENC_DELTA),
        "u16_rle": (fl.UINT16, np.repeat(rng.integers(0, 60000, n // 50 + 1), 50)[:n].astype(np.uint16), fl.ENC_RLE),
        "i8_dict": (fl.INT8, rng.choice(np.array([-7, 3, 100], dtype=np.int8), n), fl.ENC_DICT),
        "dbl": (fl.DOUBLE, np.round(rng.random(n) * 1000, 2), fl.ENC_ALP),
        "s_dict": (fl.VARCHAR, [["AIR", "MAIL", "SHIP", ""][i] for i in rng.integers(0, 4, n)], fl.ENC_DICT),
        "s_fsst": (fl.VARCHAR, [("comment %d " % i) * (i % 4) for i in range(n)], fl.ENC_FSST),
        "all_null": (fl.INT64, np.arange(n, dtype=np.int64), fl.ENC_AUTO),
        "no_null": (fl.INT32, np.arange(n, dtype=np.int32), fl.ENC_AUTO),
        "b": (fl.BOOLEAN, (rng.random(n) < 0.5).astype(np.uint8), fl.ENC_FFOR),
    }
    cols = []
    for name, (ty, vals, enc) in base.items():
        v = valid[name]
        if ty in (fl.VARCHAR, fl.BLOB):
            vv = [x if ok else None for x, ok in zip(vals, v)]
        else:
            vv = np.ma.array(vals, mask=~v)
        if name == "no_null":
            vv = vals
        cols.append((name, ty, vv, enc))
    return fl.write_image(cols, rowgroup=rowgroup), cols, valid, base


def _valid_values(fl, rf, c, ty):
    if ty in (fl.VARCHAR, fl.BLOB):
        return rf.strings_column(c)
    return np.concatenate([rf.decode(c, g) for g in range(rf.nrowgroups)]).view(fl.NP_DTYPE[ty])


@pytest.mark.parametrize("n,rowgroup", [(1, 65536), (3000, 1024), (70000, 65536)])
def test_writer_stores_validity_and_oracle_reads_it_cpu(fl, ref, n, rowgroup):
    img, cols, valid, base = _nullable_table(fl, n, 11 + n, rowgroup)
    rf = ref.RefFile(img)
    for c, (name, ty, _, _) in enumerate(cols):
        got_valid = rf.valid_column(c)
        assert np.array_equal(got_valid, valid[name]), name
        if name == "no_null":
            assert all(rf.validity(c, g) is None for g in range(rf.nrowgroups))
        vals = _valid_values(fl, rf, c, ty)
        exp = base[name][1]
        for i in np.nonzero(valid[name])[0][:: max(1, n // 5000)]:
            if ty in (fl.VARCHAR, fl.BLOB):
                assert vals[i] == exp[i].encode(), (name, i)
            elif ty == fl.DOUBLE:
                assert vals[i] == exp[i] or (np.isnan(vals[i]) and np.isnan(exp[i])), (name, i)
            else:
                assert vals[i] == exp[i], (name, i)


def test_null_placeholders_are_free_to_encode_cpu(fl, ref):
    """A NULL row holds the previous valid value (strings: ''), so sparse
    NULLs do not widen FFOR and keep DELTA/RLE runs: the nullable column's
    chunk is no larger than the same values without NULLs plus its bitmaps."""
    n = 65536
    rng = np.random.default_rng(5)
    vals = rng.integers(0, 16, n).astype(np.int32)
    mask = rng.random(n) < 0.2
    plain = fl.write_image([("a", fl.INT32, vals, fl.ENC_FFOR)])
    nullable = fl.write_image([("a", fl.INT32, np.ma.array(vals, mask=mask), fl.ENC_FFOR)])
    assert nullable.len <= plain.len + 64 * 128 + 16
    rf = ref.RefFile(nullable)
    got = rf.decode(0, 0).view(np.int32)
    assert np.array_equal(got[~mask], vals[~mask])
    assert got.max() < 16 and got.min() >= 0


def test_zone_maps_carry_null_flags_cpu(fl):
    """Zone maps are over the valid rows: ZM_HAS_NULL (8) when a row is NULL,
    ZM_ALL_NULL (16) without ZM_VALID when every row is (fls_table_zonemap)."""
    n = 5000
    vals = np.arange(n, dtype=np.int64) + 100
    m = np.zeros(n, dtype=bool)
    m[:10] = True                                   # the minimum rows are NULL
    img = fl.write_image([("a", fl.INT64, np.ma.array(vals, mask=m), fl.ENC_FFOR),
                          ("z", fl.INT64, np.ma.array(vals, mask=np.ones(n, bool)), fl.ENC_FFOR),
                          ("s", fl.VARCHAR, [None] + ["x"] * (n - 1), fl.ENC_DICT)])
    t = fl.Connection([0]).read_image(img)
    mn, mx, fl_a = t.zonemap(0, 0)
    assert (mn, mx) == (110, n + 99) and fl_a & 8 and fl_a & 1
    _, _, fl_z = t.zonemap(0, 1)
    assert fl_z == 8 | 16
    assert t.zonemap(0, 2)[2] == 8
    # pruning: IS NULL needs a NULL, IS NOT NULL and comparisons a valid row
    assert t.may_match(0, [(0, "is_null", None)]) and t.may_match(0, [(1, "is_null", None)])
    assert not t.may_match(0, [(1, "is_not_null", None)]) and not t.may_match(0, [(1, ">", 0)])
    assert not t.may_match(0, [(0, "<", 110)]) and t.may_match(0, [(0, "<=", 110)])
    w = t.validity(0, 0)
    assert w is not None and w[0] == ~np.uint64(1023) and t.validity(0, 2)[0] == ~np.uint64(1)


@pytest.mark.gpu
@pytest.mark.parametrize("n,rowgroup", [(3000, 1024), (70000, 65536)])
def test_gpu_decode_of_nullable_chunks_matches_oracle(fl, ref, gpu, n, rowgroup):
    """The HIP decode of chunks carrying bitmaps is bit-identical to the
    oracle's, placeholders included (the bitmaps sit after the encoded data)."""
    from helpers import assert_column_equal, gpu_decode_all
    img, cols, valid, base = _nullable_table(fl, n, 21 + n, rowgroup)
    t, st, out = gpu_decode_all(fl, img)
    rf = ref.RefFile(img)
    for c in range(len(cols)):
        assert_column_equal(fl, rf, c, out[c], img.ptr)


def _rows_of(fl, t, cols, filt=None):
    """(global row, valid per column, values per column) of a C-ABI scan"""
    t.set_filter(filt or [])
    rows, vals, oks = [], [[] for _ in cols], [[] for _ in cols]
    sch = t.schema()
    for first, arrays, valids, sel in t.scan_nulls():
        idx = np.arange(len(arrays[0]) // sch[0][4]) if sel is None else sel
        rows += (first + idx).tolist() if sel is None else (first + sel.astype(np.int64)).tolist()
        for c in range(len(cols)):
            ok = valids[c] if valids[c] is not None else np.ones(len(idx), dtype=bool)
            oks[c].append(ok)
            vals[c].append(arrays[c])
    return rows, [np.concatenate(o) if o else np.zeros(0, bool) for o in oks], vals


@pytest.mark.gpu
@pytest.mark.parametrize("rowgroup", [1024, 65536])
def test_scan_delivers_validity_unfiltered_and_filtered(fl, gpu, rowgroup):
    """fls_rowgroup.validity: every delivered row's NULL-ness, for a full
    scan (the image's bitmaps) and for filtered scans (gathered through sel);
    IS NULL / IS NOT NULL / comparisons select exactly DuckDB's rows (a NULL
    satisfies no comparison)."""
    n = 70000
    img, cols, valid, base = _nullable_table(fl, n, 5, rowgroup)
    names = [c[0] for c in cols]
    t = fl.Connection([0]).read_image(img)
    rows, oks, _ = _rows_of(fl, t, cols)
    assert rows == list(range(n))
    for c, name in enumerate(names):
        assert np.array_equal(oks[c], valid[name]), name
    i32 = names.index("i32")
    v = base["i32"][1]
    cases = [
        ([(i32, "is_null", None)], ~valid["i32"]),
        ([(i32, "is_not_null", None)], valid["i32"]),
        ([(i32, ">", 500)], valid["i32"] & (v > 500)),
        ([(i32, "<", -900), (i32, "is_null", None)], np.zeros(n, bool)),
        ([(i32, "<", -900, 7), (i32, "is_null", None, 7)], (valid["i32"] & (v < -900)) | ~valid["i32"]),
        ([(names.index("all_null"), "is_not_null", None)], np.zeros(n, bool)),
        ([(names.index("s_dict"), "=", "AIR")], valid["s_dict"] & (np.array(base["s_dict"][1]) == "AIR")),
        ([(names.index("s_dict"), "=", "")], valid["s_dict"] & (np.array(base["s_dict"][1]) == "")),
    ]
    for filt, exp in cases:
        rows, oks, _ = _rows_of(fl, t, cols, filt)
        assert rows == np.nonzero(exp)[0].tolist(), filt
        for c, name in enumerate(names):
            assert np.array_equal(oks[c], valid[name][rows]), (filt, name)
    t.set_filter([])


def _shortest_g(t):
    """the harness's DOUBLE -> VARCHAR rendering: the shortest %g that reads back"""
    x = float(t)
    for p in range(1, 18):
        r = "%.*g" % (p, x)
        if float(r) == x:
            return r
    return repr(x)


def _nullable_values(n, seed):
    """COPY ... VALUES columns with NULLs (cells as text, None = NULL) and the
    text DuckDB renders for each cell"""
    rng = np.random.default_rng(seed)
    null = rng.random((8, n)) < np.array([[0.1], [0.02], [0.3], [0.25], [0.5], [0.2], [0.15], [1.0]])
    null[0, :7] = True
    if n > 3000:
        null[1, 2048:4096] = True              # whole vectors
    days = rng.integers(8000, 11000, n)
    cols = [
        ("i", "INTEGER", [str((i * 7919) % 100003 - 50000) for i in range(n)]),
        ("big", "BIGINT", [str(i * 1000003) for i in range(n)]),
        ("d", "DOUBLE", [repr(float(i) / 4) for i in range(n)]),
        ("s", "VARCHAR", [f"v{i % 11}" * (i % 6) for i in range(n)]),
        ("b", "BOOLEAN", ["true" if i % 3 else "false" for i in range(n)]),
        ("x", "BLOB", [bytes([i % 256, 0, 255])[: i % 4].hex() for i in range(n)]),
        ("m", "DECIMAL(9,2)", ["%d.%02d" % (i // 7, i % 100) for i in range(n)]),
        ("z", "BIGINT", ["1"] * n),
    ]
    shown = {
        "i": lambda t: t, "big": lambda t: t, "s": lambda t: t, "b": lambda t: t, "z": lambda t: t,
        "d": _shortest_g,
        "x": lambda t: "".join(chr(c) if 32 <= c <= 126 and chr(c) not in "\\'\"" else "\\x%02X" % c
                               for c in bytes.fromhex(t)),
        "m": lambda t: t,
    }
    out_cols, expect = [], []
    for k, (name, ty, cells) in enumerate(cols):
        vals = [None if null[k, i] else cells[i] for i in range(n)]
        out_cols.append((name, ty, vals))
        expect.append([None if v is None else shown[name](v) for v in vals])
    out_cols.append(("row", "BIGINT", [str(i) for i in range(n)]))
    expect.append([str(i) for i in range(n)])
    return out_cols, [list(r) for r in zip(*expect)], null


@pytest.mark.gpu
@pytest.mark.parametrize("threads", [1, 3])
def test_copy_nulls_round_trip_through_read_fastlanes(ext, gpu, tmpfile, threads):
    """a COPY of a NULL-bearing table round-trips through
    read_fastlanes on the GPU -- every cell, NULL or value, and the types."""
    n = 3 * 4096 + 321
    cols, expect, _ = _nullable_values(n, threads)
    dst = tmpfile(f"rt{threads}.fls")
    assert ext.copy_values(cols, dst, threads=threads, row_group_size=4096) == n
    names, types, rows = ext.query("read_fastlanes", dst, threads=threads)
    assert names == [c[0] for c in cols]
    assert types == ["INTEGER", "BIGINT", "DOUBLE", "VARCHAR", "BOOLEAN", "BLOB", "DECIMAL(9,2)", "BIGINT", "BIGINT"]
    rows.sort(key=lambda r: int(r[-1]))
    for i in range(n):
        assert rows[i] == expect[i], (i, rows[i], expect[i])
    # and once more through COPY (SELECT * FROM read_fastlanes(..)): DuckDB vectors with validity in
    again = tmpfile(f"rt{threads}_2.fls")
    assert ext.copy("read_fastlanes", dst, again, threads=threads, row_group_size=4096) == n
    _, _, rows2 = ext.query("read_fastlanes", again)
    rows2.sort(key=lambda r: int(r[-1]))
    assert rows2 == rows


@pytest.mark.gpu
@pytest.mark.parametrize("threads", [1, 2])
def test_null_filters_through_read_fastlanes(ext, gpu, tmpfile, threads):
    """IS NULL / IS NOT NULL / comparisons pushed into read_fastlanes select
    DuckDB's rows: a NULL satisfies IS NULL and nothing else."""
    n = 2 * 4096 + 99
    cols, expect, null = _nullable_values(n, 7)
    dst = tmpfile("nf.fls")
    assert ext.copy_values(cols, dst, row_group_size=4096) == n
    ivals = [int(x) for x in cols[0][2] if x is not None]
    cases = [
        ([(0, "ISNULL")], lambda i: null[0, i]),
        ([(0, "ISNOTNULL")], lambda i: not null[0, i]),
        ([(0, "> 0")], lambda i: not null[0, i] and int(cols[0][2][i]) > 0),
        ([(3, "= ")], lambda i: not null[3, i] and cols[3][2][i] == ""),
        ([(4, "= true"), (1, "ISNULL")], lambda i: not null[4, i] and cols[4][2][i] == "true" and null[1, i]),
        ([(7, "ISNOTNULL")], lambda i: False),
        ([(7, "ISNULL")], lambda i: True),
    ]
    assert ivals
    for where, keep in cases:
        _, _, rows = ext.query("read_fastlanes", dst, where=where, threads=threads)
        got = sorted(int(r[-1]) for r in rows)
        assert got == [i for i in range(n) if keep(i)], where
        for r in rows:
            assert r == expect[int(r[-1])]


@pytest.mark.gpu
def test_nulls_through_scan_fastlanes_and_facade(ext, gpu, tmpfile):
    """scan_fastlanes renders a NULL cell as NULL (the reference's monostate
    column, src/fastlanes_facade.cpp:113-117) and the typed facade read API
    boxes it as a NULL Value."""
    n = 3000
    cols, expect, null = _nullable_values(n, 3)
    dst = tmpfile("sf.fls")
    assert ext.copy_values(cols, dst) == n
    _, _, rows = ext.query("scan_fastlanes", dst)
    assert rows == [[e[0]] for e in expect]
    _, _, frows, _ = ext.facade_read(dst)
    assert frows == expect
