"""Narrowed delivery (fls_scan_narrow): integer, DATE and DECIMAL columns
cross PCIe as value - (their row group's zone-map minimum) in 1, 2 or 4
bytes, and the consumer adds the base back (read_fastlanes: while filling
DuckDB's vectors).  The delivered values must be byte-identical to the full
width delivery, filtered or not, NULL placeholders included."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _scan(t, narrow, filt=None):
    t.set_filter(filt or [])
    t.narrow(narrow)
    out = None
    for first, arrays in t.scan():
        if out is None:
            out = [[] for _ in arrays]
        for c, a in enumerate(arrays):
            out[c].append(a)
    t.narrow(False)
    t.set_filter([])
    return [np.concatenate(x) if x else np.zeros(0, np.uint8) for x in out]


@pytest.mark.parametrize("wl,filt", [("lineitem", None), ("lineitem", [(10, ">=", 9000)]),
                                     ("lineitem_full", None)])
def test_narrowed_scan_matches_full_width(fl, gpu, wl, filt):
    t = fl.Connection([0]).read_image(fl.gen_image(wl, 0.02))
    full = _scan(t, False, filt)
    nar = _scan(t, True, filt)
    sch = t.schema()
    for c in range(t.ncols):
        if sch[c][1] in (fl.VARCHAR, fl.BLOB):
            continue  # string_t records: pointers compared by content elsewhere
        assert np.array_equal(full[c], nar[c]), sch[c][0]


def _scan_strings(fl, t, narrow, threads_cols):
    """string columns decoded to bytes while each row group is held (the
    records point into the scan's pinned heaps)"""
    t.set_filter([])
    t.narrow(narrow)
    out = {c: [] for c in threads_cols}
    for first, arrays in t.scan():
        for c in threads_cols:
            out[c] += fl.string_t_decode(arrays[c])
    t.narrow(False)
    return out


@pytest.fixture
def strlen_on(monkeypatch):
    monkeypatch.setenv("FLS_SCAN_STRLEN", "1")   # FSST-as-lengths delivery (the default since round 4)


def test_fsst_records_delivery_when_lengths_off(fl, gpu, monkeypatch):
    """FLS_SCAN_STRLEN=0: a narrowed scan ships the GPU-built string_t records
    (round 3's delivery); the strings equal the full-width scan's"""
    monkeypatch.setenv("FLS_SCAN_STRLEN", "0")
    t = fl.Connection([0]).read_image(fl.gen_image("lineitem_full", 0.02))
    sch = t.schema()
    sc = [c for c in range(t.ncols) if sch[c][0] == "l_comment"]
    full = _scan_strings(fl, t, False, sc)
    nar = _scan_strings(fl, t, True, sc)
    for c in sc:
        assert len(full[c]) == t.nrows and full[c] == nar[c]


@pytest.mark.parametrize("scale", [0.02, 0.25])
def test_fsst_lengths_delivery_matches_records(fl, gpu, strlen_on, scale):
    """FSST columns cross PCIe as string lengths when narrowed (unfiltered
    scans) and their string_t records are rebuilt on the host over the pinned
    heap: every string equals the one the GPU-built records give, inline
    (<= 12 bytes) and pointer records alike; the row group reports string_t
    (not narrowed, 16 bytes per value)"""
    import ctypes as C
    t = fl.Connection([0]).read_image(fl.gen_image("lineitem_full", scale))
    sch = t.schema()
    sc = [c for c in range(t.ncols) if sch[c][0] == "l_comment"]
    full = _scan_strings(fl, t, False, sc)
    nar = _scan_strings(fl, t, True, sc)
    for c in sc:
        assert len(full[c]) == t.nrows and full[c] == nar[c]
        assert full[c][:3] == fl.gen_strings("lineitem_full", c, 0, 3, scale=scale)
    t.narrow(True)
    fl._check(fl.lib.fls_scan_begin(t.h, None, 0, t.nrowgroups))
    rg = fl.RowGroup()
    assert fl._check(fl.lib.fls_scan_next(t.h, C.byref(rg))) == 1
    assert (rg.narrow[sc[0]], rg.dict_width[sc[0]]) == (0, 16)
    t.narrow(False)


def test_fsst_lengths_deferred_records(fl, gpu, strlen_on):
    """fls_scan_defer_records: acquire hands the row group out without its
    records; fls_scan_build_records (the consumer, outside its own lock)
    builds them -- the same strings as the immediate build"""
    import ctypes as C
    t = fl.Connection([0]).read_image(fl.gen_image("lineitem_full", 0.02))
    c = [k for k in range(t.ncols) if t.schema()[k][0] == "l_comment"][0]
    want = _scan_strings(fl, t, False, [c])[c]
    t.narrow(True)
    fl._check(fl.lib.fls_scan_defer_records(t.h, 1))
    fl._check(fl.lib.fls_scan_begin(t.h, None, 0, t.nrowgroups))
    rg = fl.RowGroup()
    got = []
    while fl._check(fl.lib.fls_scan_acquire(t.h, C.byref(rg))) == 1:
        fl._check(fl.lib.fls_scan_build_records(t.h, C.byref(rg)))
        p = C.cast(rg.columns[c], C.POINTER(C.c_uint8))
        got += fl.string_t_decode(np.ctypeslib.as_array(p, shape=(16 * rg.nrows,)).copy())
        fl._check(fl.lib.fls_scan_release(t.h, rg.rowgroup))
    assert fl.lib.fls_scan_build_records(t.h, C.byref(rg)) < 0   # not held any more
    fl._check(fl.lib.fls_scan_defer_records(t.h, 0))
    t.narrow(False)
    assert got == want


def test_fsst_lengths_short_and_long_strings(fl, gpu, strlen_on):
    """lengths of 1, 2 and 4 bytes (strings up to 255, 65535 and beyond),
    empty strings and NULLs, each column through the host-built records"""
    rng = np.random.default_rng(11)
    n = 2 * 65536 + 500
    words = [b"ab", b"xyz", b"0123456789", b"", b"q" * 13]
    short = [b"".join(words[j] for j in rng.integers(0, 5, rng.integers(0, 6))) for _ in range(n)]
    mid = [(b"m" * int(rng.integers(0, 700))) if i % 97 == 0 else short[i] for i in range(n)]
    big = [(b"B" * 70000) if i == 5 else short[i] for i in range(n)]
    nul = [None if i % 7 == 0 else short[i] for i in range(n)]
    cols = [("s", fl.VARCHAR, short, fl.ENC_FSST), ("m", fl.VARCHAR, mid, fl.ENC_FSST),
            ("b", fl.BLOB, big, fl.ENC_FSST), ("n", fl.VARCHAR, nul, fl.ENC_FSST)]
    t = fl.Connection([0]).read_image(fl.write_image(cols))
    full = _scan_strings(fl, t, False, range(4))
    nar = _scan_strings(fl, t, True, range(4))
    for c, (_, _, vals, _) in enumerate(cols):
        assert nar[c] == full[c]
        assert nar[c] == [b"" if v is None else v for v in vals]


def test_narrowed_widths_used(fl, gpu):
    """lineitem's DECIMAL / DATE / small-range columns do go narrow"""
    import ctypes as C
    t = fl.Connection([0]).read_image(fl.gen_image("lineitem", 0.02))
    t.narrow(True)
    fl._check(fl.lib.fls_scan_begin(t.h, None, 0, t.nrowgroups))
    rg = fl.RowGroup()
    assert fl._check(fl.lib.fls_scan_next(t.h, C.byref(rg))) == 1
    widths = {t.column(c).name.decode(): (rg.narrow[c], rg.dict_width[c]) for c in range(t.ncols)}
    assert widths["l_quantity"] == (1, 2) and widths["l_discount"] == (1, 1) and widths["l_tax"] == (1, 1)
    assert widths["l_shipdate"][0] == 1 and widths["l_shipdate"][1] == 2
    assert widths["l_returnflag"][0] == 0       # strings are never narrowed
    t.narrow(False)


def test_narrowed_nullable_and_negative(fl, gpu):
    """signed ranges around zero, NULL placeholders and all-NULL chunks"""
    rng = np.random.default_rng(3)
    n = 3 * 65536 + 99
    a = rng.integers(-1000, 1000, n).astype(np.int32)
    b = (rng.integers(0, 1 << 20, n) - (1 << 40)).astype(np.int64)
    m = rng.random(n) < 0.2
    z = np.ma.array(np.arange(n, dtype=np.int64), mask=np.ones(n, bool))
    img = fl.write_image([("a", fl.INT32, np.ma.array(a, mask=m), fl.ENC_FFOR), ("b", fl.INT64, b, fl.ENC_AUTO),
                          ("z", fl.INT64, z, fl.ENC_FFOR)])
    t = fl.Connection([0]).read_image(img)
    for filt in (None, [(0, ">", 0)], [(0, "is_null", None)]):
        full = _scan(t, False, filt)
        nar = _scan(t, True, filt)
        for c in range(3):
            assert np.array_equal(full[c], nar[c]), (filt, c)


@pytest.mark.parametrize("wl", ["lineitem", "lineitem_full"])
def test_read_fastlanes_narrowed_checksum(fl, gpu, tmpfile, wl):
    """read_fastlanes narrows at >= 4 scan threads (ReadInitGlobal): its
    DataChunks hash the same as the 1-thread (full-width) scan, every value
    of every column (the harness checksum is thread-count independent), with
    and without a pushed-down filter."""
    import sys
    sys.path.insert(0, str(__import__("pathlib").Path(__file__).parent))
    from ext_harness import Ext
    p = tmpfile(f"{wl}.fls")
    fl.gen_image(wl, 0.02).write(p)
    e = Ext()
    try:
        one = e.scan_count("read_fastlanes", p, threads=1)
        many = e.scan_count("read_fastlanes", p, threads=4)
        assert one[:2] == many[:2]
        w1 = e.scan_count("read_fastlanes", p, threads=1, where=[(4, "< 24")])
        w4 = e.scan_count("read_fastlanes", p, threads=4, where=[(4, "< 24")])
        assert w1[:2] == w4[:2] and 0 < w1[0] < one[0]
    finally:
        e.close()
