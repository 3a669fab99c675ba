"""Filter pushdown and row-group pruning -- SURVEY.md 8(f) row 4.

The reference registers its scanner with filter_pushdown = false
(src/scanner/scan_fastlanes.cpp:154): DuckDB decodes every row and filters on
the CPU.  read_fastlanes pushes DuckDB's TableFilterSet into the engine
(fls_scan_filter): zone maps and DICT dictionaries prune whole row groups on
the host, the GPU evaluates the filter per row over the decoded batch and only
qualifying rows are compacted into pinned host memory.

Oracle: the generators' ground truth (lossless, so the expected rows are a
pure function of seed and row) filtered by a numpy restatement of DuckDB's
comparison semantics (tests/helpers.py filter_mask).  Parity unpinned at the
FastLanes byte level, as for the rest of the format.

CPU tests: zone maps, pruning decisions (conservative everywhere, exact on
sorted keys and dictionaries), the TableFilter -> predicate conversion's
error paths.  GPU tests: filtered scans through the C-ABI and through
read_fastlanes' table function, bit-exact against the oracle."""
import numpy as np
import pytest

from ext_harness import Ext
from helpers import filter_mask

SF = 0.1
WL = "lineitem"
DAY_1994, DAY_1995 = 8766, 9131       # 1994-01-01, 1995-01-01 as DATE days
C_OKEY, C_PART, C_LINE, C_QTY, C_PRICE, C_DISC = 0, 1, 3, 4, 5, 6
C_RFLAG, C_SHIPDATE, C_INSTRUCT, C_MODE = 8, 10, 13, 14


@pytest.fixture(scope="module")
def lineitem(fl):
    img = fl.gen_image(WL, SF)
    conn = fl.Connection([0])
    t = conn.read_image(img)
    n = t.nrows
    sch = t.schema()
    cols = {}
    for c, (name, ty, _, _, _) in enumerate(sch):
        if ty == fl.VARCHAR:
            codes = fl.gen_values(WL, c, 0, n, np.uint32, SF)
            words = []
            while (s := fl.gen_dict_string(WL, c, len(words))) is not None:
                words.append(s.encode())
            cols[c] = [words[k] for k in codes]
        else:
            cols[c] = fl.gen_values(WL, c, 0, n, fl.NP_DTYPE[ty], SF)
    return img, t, cols


@pytest.fixture(scope="module")
def ext(_built):
    e = Ext()
    yield e
    e.close()


def rg_slice(cols, rg, rows=65536):
    return {c: v[rg * rows:(rg + 1) * rows] for c, v in cols.items()}


Q6 = [(C_SHIPDATE, ">=", DAY_1994), (C_SHIPDATE, "<", DAY_1995), (C_DISC, ">=", 5), (C_DISC, "<=", 7),
      (C_QTY, "<", 2400)]
PREDICATES = {
    "q6": Q6,
    "okey_range": [(C_OKEY, ">=", 30000), (C_OKEY, "<", 130000)],
    "mode_in": [(C_MODE, "=", "AIR", 1), (C_MODE, "=", "MAIL", 1), (C_LINE, "<=", 2)],
    "long_string": [(C_INSTRUCT, "=", "DELIVER IN PERSON")],
    "string_range": [(C_INSTRUCT, ">", "COLLECT COD"), (C_INSTRUCT, "<=", "NONE"), (C_RFLAG, "!=", "N")],
    "string_prefix_tie": [(C_INSTRUCT, "<", "TAKE BACK RETURNZ"), (C_INSTRUCT, ">=", "TAKE")],
    "nothing": [(C_PART, "<", 0)],
    "or_across_columns": [(C_LINE, "=", 7, 5), (C_DISC, "=", 0, 5)],
    "is_null": [(C_PART, "is_null", None)],
    "is_not_null": [(C_PART, "is_not_null", None), (C_PRICE, ">", 9000000)],
}


# ---------------------------------------------------------------- CPU tests
def test_zonemaps_match_generator(fl, lineitem):
    img, t, cols = lineitem
    sch = t.schema()
    for rg in range(t.nrowgroups):
        part = rg_slice(cols, rg)
        for c, (name, ty, *_) in enumerate(sch):
            z = t.zonemap(rg, c)
            if ty == fl.VARCHAR:
                assert z is None, name
                continue
            assert z is not None, name
            assert (z[0], z[1]) == (int(part[c].min()), int(part[c].max())), (name, rg)


def test_zonemaps_float_nan_and_unsigned(fl):
    d = np.array([1.5, np.nan, -2.0, -0.0, 7.25] * 300)
    f = np.array([np.nan] * 1500, dtype=np.float32)
    u = np.array([2**63 + 5, 3, 2**64 - 1] * 500, dtype=np.uint64)
    img = fl.write_image([("d", fl.DOUBLE, d, fl.ENC_AUTO), ("f", fl.FLOAT, f, fl.ENC_AUTO),
                          ("u", fl.UINT64, u, fl.ENC_AUTO)], rowgroup=1024)
    t = fl.Connection([0]).read_image(img)
    lo, hi, flags = t.zonemap(0, 0)
    assert (lo, hi) == (-2.0, 7.25) and flags & 2 and not flags & 4
    assert t.zonemap(0, 1)[2] & 4                       # all NaN
    assert t.zonemap(0, 2)[:2] == (3, 2**64 - 1)         # unsigned order
    assert t.may_match(0, [(0, "=", float("nan"))])      # NaN present
    assert t.may_match(0, [(0, ">", 7.25)])             # NaN > 7.25 in DuckDB order
    assert t.may_match(0, [(1, ">", 1e30)])              # all-NaN chunk: NaN > everything
    assert not t.may_match(0, [(1, "<", 1e30)])
    assert not t.may_match(0, [(2, "<", 3)])
    assert t.may_match(0, [(2, ">", 2**63)])


@pytest.mark.parametrize("name", sorted(PREDICATES))
def test_pruning_is_conservative(fl, lineitem, name):
    img, t, cols = lineitem
    terms = PREDICATES[name]
    for rg in range(t.nrowgroups):
        part = rg_slice(cols, rg)
        n = t.rowgroup_rows(rg)
        if not t.may_match(rg, terms):
            assert not filter_mask(part, terms, n).any(), (name, rg)


def test_pruning_exact_on_sorted_keys_and_dictionaries(fl, lineitem):
    img, t, cols = lineitem
    okey = cols[C_OKEY]
    for k0, k1 in [(30000, 130000), (1, 2), (okey[-1], okey[-1] + 1), (10**9, 10**9 + 5)]:
        terms = [(C_OKEY, ">=", int(k0)), (C_OKEY, "<", int(k1))]
        for rg in range(t.nrowgroups):
            hit = filter_mask(rg_slice(cols, rg), terms, t.rowgroup_rows(rg)).any()
            assert t.may_match(rg, terms) == hit, (k0, k1, rg)   # keys sorted: zone maps are exact
    assert not any(t.may_match(rg, [(C_MODE, "=", "BOAT")]) for rg in range(t.nrowgroups))
    assert all(t.may_match(rg, [(C_MODE, "=", "BOAT", 1), (C_MODE, "=", "RAIL", 1)]) for rg in range(t.nrowgroups))
    assert not t.may_match(0, [(C_PART, "is_null", None)])


def test_filter_argument_errors(fl, lineitem):
    img, t, cols = lineitem
    with pytest.raises(fl.FlsError, match="out of range"):
        t.set_filter([(99, "=", 1)])
    t.set_filter([])


def test_read_fastlanes_unsupported_filter_shape(fl, ext, tmpfile):
    """A shape the engine cannot evaluate (an optional filter inside an OR)
    used to fail the query with NotImplementedException; it now binds and is
    applied on the host (the optional branch conservatively true: DuckDB
    re-checks optional filters above the scan)."""
    p = tmpfile("li.fls")
    fl.gen_image(WL, 0.01).write(p)
    names, _, rows = ext.query("read_fastlanes", p, proj=[0], limit=0, where=[(C_LINE, "OR OPT = 1|= 2")])
    assert names == ["l_orderkey"] and rows == []


@pytest.mark.gpu
def test_read_fastlanes_unsupported_filter_shape_rows(fl, ext, gpu, tmpfile):
    p = tmpfile("li.fls")
    fl.gen_image(WL, 0.01).write(p)
    _, _, rows = ext.query("read_fastlanes", p, proj=[0], where=[(C_LINE, "OR OPT = 1|= 2")])
    assert len(rows) == fl.gen_nrows(WL, 0.01)   # a superset, never fewer rows than the filter keeps


# ---------------------------------------------------------------- GPU tests
def check_filtered_scan(fl, t, cols, terms, deliver):
    """Engine-level filtered scan vs the oracle, per row group: selection and
    delivered values bit-exact; pruned row groups never delivered."""
    sch = t.schema()
    expect_pruned = sum(not t.may_match(rg, terms) for rg in range(t.nrowgroups))
    seen = set()
    total = 0
    for rg, first_row, sel, arrays in t.scan_filtered(terms, cols=deliver):
        seen.add(rg)
        part = rg_slice(cols, rg)
        n = t.rowgroup_rows(rg)
        want = np.nonzero(filter_mask(part, terms, n))[0]
        assert np.array_equal(sel, want), (rg, len(sel), len(want))
        total += len(sel)
        for c in deliver:
            ty = sch[c][1]
            if ty == fl.VARCHAR:
                assert fl.string_t_decode(arrays[c]) == [part[c][i] for i in want], (sch[c][0], rg)
            else:
                assert np.array_equal(arrays[c].view(fl.NP_DTYPE[ty]), part[c][want]), (sch[c][0], rg)
    assert t.pruned == expect_pruned
    assert len(seen) == t.nrowgroups - expect_pruned
    return total


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(PREDICATES))
def test_gpu_filtered_scan_bit_exact(fl, gpu, lineitem, name):
    img, t, cols = lineitem
    terms = PREDICATES[name]
    deliver = [C_OKEY, C_PRICE, C_SHIPDATE, C_INSTRUCT, C_MODE]
    total = check_filtered_scan(fl, t, cols, terms, deliver)
    assert total == int(filter_mask(cols, terms, t.nrows).sum())


@pytest.mark.gpu
@pytest.mark.parametrize("batch", ["1", "3"])
def test_gpu_filtered_scan_batches_and_filter_only_columns(fl, gpu, lineitem, monkeypatch, batch):
    # filter columns not delivered (decoded on the GPU only); odd batch sizes
    # make batches end mid-run of surviving row groups
    monkeypatch.setenv("FLS_SCAN_BATCH", batch)
    img, t, cols = lineitem
    terms = [(C_OKEY, ">=", 40000), (C_OKEY, "<", 500000), (C_DISC, "<", 3)]
    check_filtered_scan(fl, t, cols, terms, [C_PART, C_MODE])


@pytest.mark.gpu
def test_gpu_filtered_scan_floats_nan_unsigned(fl, gpu):
    rng = np.random.default_rng(7)
    n = 70000
    pool = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1.5, -1.5, 2.25, 1e300])
    d = np.where(rng.random(n) < 0.3, pool[rng.integers(0, len(pool), n)], np.round(rng.normal(0, 10, n), 2))
    with np.errstate(over="ignore"):
        f = d.astype(np.float32)
    u = rng.integers(0, 2**64 - 1, n, dtype=np.uint64)
    i8 = rng.integers(-128, 128, n).astype(np.int8)
    img = fl.write_image([("d", fl.DOUBLE, d, fl.ENC_AUTO), ("f", fl.FLOAT, f, fl.ENC_AUTO),
                          ("u", fl.UINT64, u, fl.ENC_AUTO), ("i", fl.INT8, i8, fl.ENC_AUTO)])
    t = fl.Connection([0]).read_image(img)
    cols = {0: d, 1: f, 2: u, 3: i8}
    for terms in ([(0, "=", float("nan"))], [(0, ">", 2.0)], [(0, "<=", -0.0)], [(0, "=", 0.0)],
                  [(1, "!=", float("nan")), (1, ">=", -1.5)], [(1, ">", float("inf"))],
                  [(2, ">", 2**63)], [(2, "<=", 12345678901234)], [(3, "<", -100, 1), (3, ">", 100, 1)],
                  [(3, "=", -128)]):
        rows = []
        for rg, first_row, sel, arrays in t.scan_filtered(terms, cols=[0, 1, 2, 3]):
            rows.append(sel + rg * 65536)
            got_d = arrays[0].view(np.float64)
            exp_d = d[sel + rg * 65536]
            assert np.array_equal(got_d.view(np.uint64), exp_d.view(np.uint64)), terms
        got = np.concatenate(rows) if rows else np.zeros(0, np.int64)
        want = np.nonzero(filter_mask(cols, terms, n))[0]
        assert np.array_equal(got, want), terms


@pytest.mark.gpu
def test_gpu_filtered_scan_fsst_and_alp(fl, gpu):
    for wl, terms, deliver in [
        ("lineitem_full", [(15, ">=", "furiously"), (15, "<", "q")], [0, 15]),
        ("lineitem_full", [(15, "=", "")], [15]),
        ("lineitem_dbl", [(4, "<", 24.0), (6, ">=", 0.05), (6, "<=", 0.07)], [0, 4, 5, 6]),
    ]:
        img = fl.gen_image(wl, 0.02)
        t = fl.Connection([0]).read_image(img)
        n = t.nrows
        sch = t.schema()
        cols = {}
        for c in {x[0] for x in terms} | set(deliver):
            ty = sch[c][1]
            if ty == fl.VARCHAR:
                cols[c] = fl.gen_strings(wl, c, 0, n, 0.02)
            else:
                cols[c] = fl.gen_values(wl, c, 0, n, fl.NP_DTYPE[ty], 0.02)
        total = 0
        for rg, first_row, sel, arrays in t.scan_filtered(terms, cols=deliver):
            want = np.nonzero(filter_mask(rg_slice(cols, rg), terms, t.rowgroup_rows(rg)))[0]
            assert np.array_equal(sel, want), (wl, rg)
            total += len(sel)
            for c in deliver:
                ty = sch[c][1]
                exp = [cols[c][rg * 65536 + i] for i in want] if ty == fl.VARCHAR else cols[c][rg * 65536 + want]
                if ty == fl.VARCHAR:
                    assert fl.string_t_decode(arrays[c]) == exp, (wl, c)
                else:
                    assert np.array_equal(arrays[c].view(fl.NP_DTYPE[ty]), exp), (wl, c)
        assert total == int(filter_mask(cols, terms, n).sum()), wl


@pytest.mark.gpu
@pytest.mark.parametrize("threads", [1, 4])
def test_gpu_read_fastlanes_where_q6(fl, gpu, ext, lineitem, tmpfile, threads):
    # SELECT l_orderkey, l_extendedprice, rowid FROM read_fastlanes(f)
    #   WHERE <TPC-H Q6 predicate>  -- filter columns pruned from the output
    img, t, cols = lineitem
    p = tmpfile("li.fls")
    img.write(p)
    where = [(C_SHIPDATE, ">= 1994-01-01"), (C_SHIPDATE, "< 1995-01-01"), (C_DISC, ">= 0.05"),
             (C_DISC, "<= 0.07"), (C_QTY, "< 24")]
    names, types, rows = ext.query("read_fastlanes", p, proj=[C_OKEY, C_PRICE, -1], where=where, threads=threads)
    assert names == ["l_orderkey", "l_extendedprice", "rowid"]
    want = np.nonzero(filter_mask(cols, Q6, t.nrows))[0]
    assert len(rows) == len(want)
    assert [int(r[0]) for r in rows] == cols[C_OKEY][want].tolist()
    assert [int(r[2]) for r in rows] == want.tolist()
    price = cols[C_PRICE][want]
    assert [r[1] for r in rows[:50]] == [f"{v // 100}.{v % 100:02d}" for v in price[:50]]


@pytest.mark.gpu
def test_gpu_read_fastlanes_where_strings_in_or_and_multifile(fl, gpu, ext, tmp_path):
    a, b = tmp_path / "a.fls", tmp_path / "b.fls"
    fl.gen_image(WL, 0.01).write(str(a))
    fl.gen_image(WL, 0.02).write(str(b))
    where = [(C_MODE, "IN AIR|REG AIR"), (C_INSTRUCT, "OR = DELIVER IN PERSON|= NONE"), (C_LINE, "OPT < 3"),
             (C_PART, "ISNOTNULL")]
    names, types, rows = ext.query("read_fastlanes", str(tmp_path / "*.fls"), proj=[C_MODE, C_INSTRUCT, C_LINE],
                                   where=where)
    exp = []
    for sf in (0.01, 0.02):
        n = fl.gen_nrows(WL, sf)
        mode = fl.gen_values(WL, C_MODE, 0, n, np.uint32, sf)
        ins = fl.gen_values(WL, C_INSTRUCT, 0, n, np.uint32, sf)
        line = fl.gen_values(WL, C_LINE, 0, n, np.int32, sf)
        for i in range(n):
            m = fl.gen_dict_string(WL, C_MODE, int(mode[i]))
            s = fl.gen_dict_string(WL, C_INSTRUCT, int(ins[i]))
            if m in ("AIR", "REG AIR") and s in ("DELIVER IN PERSON", "NONE"):
                exp.append([m, s, str(line[i])])
    assert rows == exp


@pytest.mark.gpu
def test_gpu_read_fastlanes_where_everything_pruned(fl, gpu, ext, tmpfile):
    p = tmpfile("li.fls")
    fl.gen_image(WL, 0.01).write(p)
    assert ext.query("read_fastlanes", p, proj=[0], where=[(C_OKEY, "< 0")])[2] == []
    assert ext.query("read_fastlanes", p, proj=[0], where=[(C_PART, "ISNULL")])[2] == []
    n, h, _ = ext.scan_count("read_fastlanes", p, proj=[C_OKEY], where=[(C_MODE, "= SHIP")])
    assert n == int(sum(fl.gen_dict_string(WL, C_MODE, int(k)) == "SHIP"
                        for k in fl.gen_values(WL, C_MODE, 0, fl.gen_nrows(WL, 0.01), np.uint32, 0.01)))


# ---- filters the engine cannot evaluate stay correct (host-side residuals) ----
def test_unknown_filter_evaluated_on_host_without_gpu_is_bind_safe(fl, tmp_path):
    """Binding a scan with an EXPRESSION_FILTER no longer throws
    NotImplementedException: the filter is kept for the host."""
    from ext_harness import Ext
    p = str(tmp_path / "x.fls")
    fl.write_image([("a", fl.INT32, np.arange(5000, dtype=np.int32), fl.ENC_FFOR)]).write(p)
    e = Ext()
    try:
        names, types, rows = e.query("read_fastlanes", p, limit=0, where=[(0, "EXPR MOD 7 3")])
        assert names == ["a"] and rows == []
    finally:
        e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("threads", [1, 3])
def test_expression_filter_applied_on_host(fl, gpu, tmp_path, threads):
    """An EXPRESSION_FILTER (DuckDB pushes these only when asked; a real
    engine's scan must then honour them) is evaluated on the host over every
    delivered chunk, AND-ed with the engine's pushed-down predicates, also on
    a column that is filtered but not projected (filter_prune)."""
    from ext_harness import Ext
    n = 3 * 65536 + 777
    a = np.arange(n, dtype=np.int64) * 3 + 1
    b = (np.arange(n) % 1000).astype(np.int32)
    txt = [f"w{i % 97}x" for i in range(n)]
    p = str(tmp_path / "e.fls")
    fl.write_image([("a", fl.INT64, a, fl.ENC_DELTA), ("b", fl.INT32, b, fl.ENC_FFOR),
                    ("t", fl.VARCHAR, txt, fl.ENC_AUTO)]).write(p)
    e = Ext()
    try:
        _, _, rows = e.query("read_fastlanes", p, threads=threads, where=[(0, "EXPR MOD 7 3")])
        want = [i for i in range(n) if a[i] % 7 == 3]
        assert [int(r[0]) for r in rows] == [int(a[i]) for i in want]
        # host residual AND engine predicate, on the filtered-only column b
        _, _, rows = e.query("read_fastlanes", p, proj=[0], threads=threads,
                             where=[(0, "EXPR MOD 5 1"), (1, "< 300")])
        want = [i for i in range(n) if a[i] % 5 == 1 and b[i] < 300]
        assert [int(r[0]) for r in rows] == [int(a[i]) for i in want]
        # VARCHAR residual; a filter that rejects every row of some chunks
        _, _, rows = e.query("read_fastlanes", p, proj=[2, 1], threads=threads, where=[(2, "EXPR LIKE w13x")])
        want = [i for i in range(n) if txt[i] == "w13x"]
        assert [r[0] for r in rows] == ["w13x"] * len(want)
        assert [int(r[1]) for r in rows] == [int(b[i]) for i in want]
        _, _, rows = e.query("read_fastlanes", p, threads=threads, where=[(1, "EXPR MOD 1000 999999")])
        assert rows == []
    finally:
        e.close()
