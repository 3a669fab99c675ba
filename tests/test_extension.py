"""DuckDB glue (extension/) driven the way DuckDB drives table functions.

CPU tests: registration, the reference's exact error texts
(test/sql/fastlane.test:8-12, src/scan_fastlanes.cpp:30,34,42), typed schema
binding (footer only).  GPU tests: the fastlane.test result shape on a
synthetic 1024-row text file, scan_fastlanes' VARCHAR rendering of row group 0,
and read_fastlanes' typed, projected, multi-file scan vs the generators."""
import numpy as np
import pytest

from ext_harness import Ext, ExtError

TITLE = ("The FastLanes Compression Layout: Decoding >100 Billion Integers per Second with Scalar Code "
         "Azim Afroozeh CWI The Netherlands azim@cwi.")


@pytest.fixture(scope="module")
def ext(_built):
    e = Ext()
    yield e
    e.close()


def paper_lines(n=1024, hits=71, seed=3):
    """1024 non-empty lines; row 0 is the reference's first row, exactly `hits`
    rows contain 'FastLanes' (the shape of third_party/fastlanes/data/fls/data.fls)."""
    rng = np.random.default_rng(seed)
    words = ["vector", "lanes", "interleaved", "bit-packing", "SIMD", "decoding", "scalar", "layout",
             "transposed", "delta", "dictionary", "run-length", "compression", "integers", "register"]
    lines = [TITLE]
    hit_rows = set(rng.choice(np.arange(1, n), hits - 1, replace=False).tolist())
    for i in range(1, n):
        body = " ".join(words[j] for j in rng.integers(0, len(words), rng.integers(3, 25)))
        lines.append(("FastLanes " if i in hit_rows else "") + body + f" {i}")
    return lines


def test_registered_functions(ext):
    assert ext.has_function("scan_fastlanes")
    assert ext.has_function("read_fastlanes")


def test_fastlane_version_scalar(ext):
    # SELECT fastlane_version() (reference src/fastlane_extension.cpp:32-42,
    # examples/basic_usage.sql:8): the reference's constant text
    assert ext.scalar0("fastlane_version") == "FastLanes Extension v1.0.0"
    assert ext.scalar0("no_such_function") is None


def test_read_fastlanes_accepts_auto_detect(ext):
    # named parameter of the intended scanner (src/scanner/scan_fastlanes.cpp:156),
    # BOOLEAN (LogicalTypeId 2), on both the VARCHAR and the LIST(VARCHAR) overload
    assert ext.has_named_parameter("read_fastlanes", "auto_detect", 2)
    assert not ext.has_named_parameter("read_fastlanes", "no_such_option")


def test_nonexistent_file_error_verbatim(ext):
    # test/sql/fastlane.test:8-12
    with pytest.raises(ExtError, match="^Failed to open FastLanes file: nonexistent.fls$"):
        ext.query("scan_fastlanes", "nonexistent.fls", limit=0)
    with pytest.raises(ExtError, match="^Failed to open FastLanes file: nonexistent.fls$"):
        ext.query("read_fastlanes", "nonexistent.fls", limit=0)


def test_bind_argument_errors(ext):
    # through DuckDB's binder: arity mismatch fails overload resolution, an
    # INTEGER is implicitly cast to VARCHAR and then fails to open
    with pytest.raises(ExtError, match="No function matches"):
        ext.query("scan_fastlanes", "a.fls", "b.fls")
    with pytest.raises(ExtError, match="^Failed to open FastLanes file: 7$"):
        ext.query("scan_fastlanes", 7)
    # the Bind callback's own checks (src/scan_fastlanes.cpp:29-35), reached
    # when the arguments are handed over as given
    with pytest.raises(ExtError, match="^scan_fastlanes requires exactly one argument \\(file path\\)$"):
        ext.query("scan_fastlanes", "a.fls", "b.fls", raw=True)
    with pytest.raises(ExtError, match="^scan_fastlanes file path must be a string$"):
        ext.query("scan_fastlanes", 7, raw=True)


def test_corrupt_file_fails_bind(ext, tmpfile):
    p = tmpfile("bad.fls")
    open(p, "wb").write(b"FLSAMD01" + b"\0" * 100)
    with pytest.raises(ExtError, match="Failed to open FastLanes file"):
        ext.query("read_fastlanes", p, limit=0)


def test_read_fastlanes_schema_without_gpu(fl, ext, tmpfile):
    img = fl.gen_image("lineitem", 0.01)
    p = tmpfile("li.fls")
    img.write(p)
    names, types, rows = ext.query("read_fastlanes", p, limit=0)
    assert names[:3] == ["l_orderkey", "l_partkey", "l_suppkey"] and len(names) == 15
    assert types[0] == "BIGINT" and types[1] == "INTEGER" and types[4] == "DECIMAL(15,2)"
    assert types[8] == "VARCHAR" and types[10] == "DATE"
    assert rows == []
    # replacement scan: FROM 'x.fls'
    names2, types2, _ = ext.query(None, p, limit=0)
    assert names2 == names and types2 == types
    # projection pushdown binds only what is asked
    n3, t3, _ = ext.query("read_fastlanes", p, proj=[14, 0], limit=0)
    assert n3 == ["l_shipmode", "l_orderkey"] and t3 == ["VARCHAR", "BIGINT"]


@pytest.mark.gpu
def test_fastlane_test_shape(fl, ext, gpu, tmpfile):
    """test/sql/fastlane.test:15-66 on a synthetic data.fls of the same shape."""
    lines = paper_lines()
    p = tmpfile("data.fls")
    fl.write_image([("text", fl.VARCHAR, lines, fl.ENC_DICT)]).write(p)
    names, types, rows = ext.query("scan_fastlanes", p)
    assert names == ["data"] and types == ["VARCHAR"]
    data = [r[0] for r in rows]
    assert len(data) == 1024                                   # COUNT(*) = 1024
    assert sum(1 for d in data if len(d) > 0) == 1024          # LENGTH(data) > 0
    assert len(ext.query("scan_fastlanes", p, limit=5)[2]) == 5  # LIMIT 5
    assert sum(1 for d in data if "FastLanes" in d) == 71      # LIKE '%FastLanes%'
    assert min(map(len, data)) > 0 and max(map(len, data)) >= len(TITLE)
    assert ext.query("scan_fastlanes", p, limit=1)[2][0][0] == TITLE
    assert data == lines


@pytest.mark.gpu
def test_scan_fastlanes_semantics(fl, ext, gpu, tmpfile):
    # column 0, row group 0 only, integers rendered as decimal text, other
    # FastLanes variant types (here SMALLINT) as NULL -- src/fastlanes_facade.cpp
    n = 70000
    a = (np.arange(n, dtype=np.int64) * 7919 % 100003 - 50000).astype(np.int32)
    p = tmpfile("ints.fls")
    fl.write_image([("a", fl.INT32, a, fl.ENC_FFOR), ("b", fl.INT16, (a % 100).astype(np.int16), fl.ENC_AUTO)]).write(p)
    _, _, rows = ext.query("scan_fastlanes", p)
    assert len(rows) == 65536
    assert [r[0] for r in rows] == [str(int(x)) for x in a[:65536]]
    p2 = tmpfile("i16.fls")
    fl.write_image([("b", fl.INT16, (a % 100).astype(np.int16), fl.ENC_FFOR)]).write(p2)
    _, _, rows = ext.query("scan_fastlanes", p2, limit=10)
    assert all(r[0] is None for r in rows)


@pytest.mark.gpu
def test_read_fastlanes_typed_projected_multifile(fl, ext, gpu, tmpfile):
    img = fl.gen_image("lineitem", 0.01)
    p = tmpfile("li.fls")
    img.write(p)
    n = 60175
    names, types, rows = ext.query("read_fastlanes", p, proj=[14, 0, 10, 5, -1])
    assert len(rows) == n and names[-1] == "rowid"
    modes = fl.gen_values("lineitem", 14, 0, n, np.uint32, 0.01)
    okey = fl.gen_values("lineitem", 0, 0, n, np.int64, 0.01)
    ship = fl.gen_values("lineitem", 10, 0, n, np.int32, 0.01)
    price = fl.gen_values("lineitem", 5, 0, n, np.int64, 0.01)
    import datetime
    epoch = datetime.date(1970, 1, 1)
    for i in range(0, n, 997):
        r = rows[i]
        assert r[0] == fl.gen_dict_string("lineitem", 14, int(modes[i]))
        assert r[1] == str(int(okey[i]))
        assert r[2] == (epoch + datetime.timedelta(days=int(ship[i]))).isoformat()
        assert r[3] == f"{int(price[i]) // 100}.{int(price[i]) % 100:02d}"
        assert r[4] == str(i)
    # LIST(VARCHAR) overload: two files back to back
    _, _, rows2 = ext.query("read_fastlanes", p, p, as_list=True, proj=[0])
    assert len(rows2) == 2 * n and rows2[n][0] == rows2[0][0]


@pytest.mark.gpu
def test_read_fastlanes_stream_checksum_matches_oracle_rowcount(fl, ext, gpu, tmpfile):
    img = fl.gen_image("lineitem", 0.1)
    p = tmpfile("li01.fls")
    img.write(p)
    rows, h1, sec = ext.scan_count("read_fastlanes", p)
    assert rows == 600572
    rows2, h2, _ = ext.scan_count("read_fastlanes", p)
    assert (rows2, h2) == (rows, h1)   # deterministic end-to-end delivery
    print(f"read_fastlanes e2e SF0.1: {rows / sec / 1e6:.1f} M rows/s")


@pytest.mark.gpu
@pytest.mark.parametrize("threads", [2, 8])
def test_read_fastlanes_parallel_scan_keeps_order(fl, ext, gpu, tmpfile, monkeypatch, threads):
    """MaxThreads > 1 (reference: 1, src/scanner/scan_fastlanes.cpp:43-45):
    threads claim row groups through fls_scan_acquire/release, the batch index
    (row group position over all files) restores order."""
    monkeypatch.setenv("FLS_SCAN_BATCH", "2")
    img = fl.gen_image("lineitem", 0.1)            # 10 row groups
    p = tmpfile("li01.fls")
    img.write(p)
    one = ext.scan_count("read_fastlanes", p)
    many = ext.scan_count("read_fastlanes", p, threads=threads)
    assert many[:2] == one[:2] and one[0] == 600572
    # rows in order, projected, rowid included
    _, _, r1 = ext.query("read_fastlanes", p, proj=[-1, 0, 14])
    _, _, rn = ext.query("read_fastlanes", p, proj=[-1, 0, 14], threads=threads)
    assert rn == r1 and [int(r[0]) for r in rn[::4099]] == list(range(0, 600572, 4099))
    # several files, each scanned in parallel, concatenated in list order
    q = tmpfile("small.fls")
    fl.gen_image("lineitem", 0.01).write(q)
    _, _, m1 = ext.query("read_fastlanes", p, q, p, as_list=True, proj=[0, 10])
    _, _, mn = ext.query("read_fastlanes", p, q, p, as_list=True, proj=[0, 10], threads=threads)
    assert len(mn) == 2 * 600572 + 60175 and mn == m1


def test_read_fastlanes_glob_binds_sorted_files(fl, ext, tmp_path):
    # src/scanner/scan_fastlanes.cpp:151-185 (multi-file), DuckDB glob semantics
    with pytest.raises(ExtError, match='^No files found that match the pattern ".*nothing_\\*.fls"$'):
        ext.query("read_fastlanes", str(tmp_path / "nothing_*.fls"), limit=0)
    a = np.arange(3000, dtype=np.int32)
    for i in (2, 0, 1):
        fl.write_image([("v", fl.INT32, a + i * 10000, fl.ENC_FFOR)]).write(str(tmp_path / f"part_{i}.fls"))
    names, types, rows = ext.query("read_fastlanes", str(tmp_path / "part_*.fls"), limit=0)
    assert names == ["v"] and types == ["INTEGER"]


@pytest.mark.gpu
def test_read_fastlanes_glob_scans_in_name_order(fl, ext, gpu, tmp_path):
    a = np.arange(3000, dtype=np.int32)
    for i in (2, 0, 1):
        fl.write_image([("v", fl.INT32, a + i * 10000, fl.ENC_FFOR)]).write(str(tmp_path / f"part_{i}.fls"))
    _, _, rows = ext.query("read_fastlanes", str(tmp_path / "part_?.fls"), threads=4)
    assert [int(r[0]) for r in rows] == np.concatenate([a, a + 10000, a + 20000]).tolist()


def test_read_fastlanes_empty_file(fl, ext, tmpfile):
    """A file with a schema and zero row groups binds and scans to no rows
    (the scan ends before any device work, so this needs no GPU)."""
    img = fl.write_image([("a", fl.INT32, np.zeros(0, np.int32), fl.ENC_FFOR),
                          ("s", fl.VARCHAR, [], fl.ENC_AUTO)])
    p = tmpfile("empty.fls")
    img.write(p)
    names, types, rows = ext.query("read_fastlanes", p)
    assert names == ["a", "s"] and types == ["INTEGER", "VARCHAR"] and rows == []
    assert ext.scan_count("read_fastlanes", p)[0] == 0
    _, _, rows = ext.query("read_fastlanes", p, p, as_list=True)
    assert rows == []


@pytest.mark.gpu
@pytest.mark.parametrize("threads", [1, 4])
def test_read_fastlanes_zero_copy_chunks_stay_valid_when_held(fl, ext, gpu, tmpfile, monkeypatch, threads):
    """read_fastlanes hands DuckDB vectors that reference the engine's pinned
    row-group buffers (FlatVector::SetData + a RowGroupPin auxiliary).  A sink
    that keeps a reference to EVERY chunk and hashes them only after the scan
    has recycled every batch slot must see the same bytes as one that hashes
    them on arrival -- including l_comment (FSST), whose string_t records point
    into the batch's pinned heap (strings overwritten by a reused
    slot).  One row group per batch maximises slot reuse."""
    monkeypatch.setenv("FLS_SCAN_BATCH", "1")
    p = tmpfile("lif.fls")
    fl.gen_image("lineitem_full", 0.1).write(p)    # 10 row groups, 16 columns
    rows, h_live, _ = ext.scan_count("read_fastlanes", p, threads=threads)
    rows2, h_held, _ = ext.scan_hold("read_fastlanes", p, threads=threads)
    assert rows == rows2 == 600572 and h_held == h_live
    # the held bytes are the generator's (l_comment sample)
    _, _, got = ext.query("read_fastlanes", p, proj=[15], limit=5000)
    assert [r[0].encode() for r in got] == fl.gen_strings("lineitem_full", 15, 0, 5000, 0.1)


@pytest.mark.gpu
def test_read_fastlanes_delivery_rate_zero_copy(fl, ext, gpu, tmpfile):
    """DataChunk delivery without a checksum sink: reports rows/s at 1 and 8
    threads (the engine scan into pinned memory bounds it)."""
    p = tmpfile("li1.fls")
    fl.gen_image("lineitem", 1.0).write(p)
    for th in (1, 8):
        n, sec = ext.scan_rows("read_fastlanes", p, threads=th)
        assert n == 6001215
        print(f"read_fastlanes zero-copy DataChunks SF1, {th} threads: {n / sec / 1e6:.1f} M rows/s")


# ---- row a13: the typed facade's read API, and config C1 through DataChunks ----
def _expected_cells(fl, ref, img, wl, scale, n):
    """Every value of a generated table as DuckDB renders it (Value::ToString)."""
    import datetime
    rf = ref.RefFile(img)
    epoch = datetime.date(1970, 1, 1)
    cols = []
    for c in range(rf.ncols):
        name, ty, width, sc = rf.column(c)
        if ty == fl.VARCHAR:
            if wl == "lineitem_full" and name == "l_comment":
                cols.append([x.decode() for x in fl.gen_strings(wl, c, 0, n, scale)])
            else:
                codes = fl.gen_values(wl, c, 0, n, np.uint32, scale)
                lut = {}
                cols.append([lut.setdefault(int(k), fl.gen_dict_string(wl, c, int(k))) for k in codes])
        elif ty == fl.DATE:
            v = fl.gen_values(wl, c, 0, n, np.int32, scale)
            cols.append([(epoch + datetime.timedelta(days=int(x))).isoformat() for x in v])
        elif ty == fl.DECIMAL:
            v = fl.gen_values(wl, c, 0, n, np.int64, scale)
            cols.append([("-" if x < 0 else "") + f"{abs(int(x)) // 10 ** sc}.{abs(int(x)) % 10 ** sc:0{sc}d}"
                         for x in v])
        else:
            cols.append([str(int(x)) for x in fl.gen_values(wl, c, 0, n, fl.NP_DTYPE[ty], scale)])
    return [list(r) for r in zip(*cols)]


def test_facade_read_api_symbol_exported(ext):
    # the signatures are pinned at compile time (static_asserts in the harness
    # against the reference's declaration, incl. void finalizeFile())
    assert hasattr(ext.lib, "fls_ext_facade_read")
    with pytest.raises(ExtError, match="openFile failed"):
        ext.facade_read("/nonexistent/x.fls")


@pytest.mark.gpu
@pytest.mark.parametrize("wl,scale", [("lineitem", 0.02), ("lineitem_full", 0.012)])
def test_typed_facade_read_api_every_value(fl, ref, ext, gpu, tmpfile, wl, scale):
    """ext_fastlane::FastLanesFacade::openFile / getColumnTypes / getColumnNames
    / readNextChunk(vector<Value>&, idx_t&) -- the interface the reference's
    intended scanner calls (src/scanner/scan_fastlanes.cpp:82-83,126) -- over
    a multi-row-group lineitem file: every boxed value equals the generator's,
    chunks hold <= STANDARD_VECTOR_SIZE rows and never straddle a row group."""
    img = fl.gen_image(wl, scale)
    p = tmpfile(f"{wl}.fls")
    img.write(p)
    n = fl.gen_nrows(wl, scale)
    assert n > 65536                                       # >= 2 row groups
    names, types, rows, chunks = ext.facade_read(p)
    q_names, q_types, _ = ext.query("read_fastlanes", p, limit=0)
    assert names == q_names and types == q_types           # same schema as the table function binds
    assert len(rows) == n and sum(chunks) == n
    assert all(0 < k <= 2048 for k in chunks)
    bounds = np.cumsum([0] + chunks)
    assert all(not (b0 < 65536 * g < b1) for b0, b1 in zip(bounds, bounds[1:]) for g in range(1, n // 65536 + 1))
    want = _expected_cells(fl, ref, img, wl, scale, n)
    bad = [i for i in range(n) if rows[i] != want[i]]
    assert not bad, (bad[:3], rows[bad[0]], want[bad[0]])


@pytest.mark.gpu
def test_config_c1_through_read_fastlanes_datachunks(fl, ext, gpu, tmpfile):
    """BASELINE config C1 (1,000,000 INT32 rows, W=7 FFOR: 16 row groups, the
    last 16,960 rows) delivered as DuckDB DataChunks by read_fastlanes, every
    value vs the generator (the C-ABI path is test_gpu_decode.py's)."""
    img = fl.gen_image("c1")
    p = tmpfile("c1.fls")
    img.write(p)
    names, types, rows = ext.query("read_fastlanes", p)
    assert len(names) == 1 and types == ["INTEGER"]
    want = fl.gen_values("c1", 0, 0, 1000000, np.int32)
    assert len(rows) == 1000000
    got = np.array([int(r[0]) for r in rows], dtype=np.int64)
    assert np.array_equal(got, want.astype(np.int64))
    assert 1000000 - 15 * 65536 == 16960
    r2, h2, _ = ext.scan_count("read_fastlanes", p)
    r3, h3, _ = ext.scan_count("read_fastlanes", p, threads=4)   # parallel scan, batch-index order
    assert r2 == r3 == 1000000 and h2 == h3
