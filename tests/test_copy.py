"""COPY ... TO 'x.fls' (FORMAT fls | fastlane) -- SURVEY.md 8(f) row 1.

The reference carries this writer uncompiled (src/writer/write_fastlane_stream.cpp:
65-314: options ROW_GROUP_SIZE / CHUNK_SIZE default 65,536, ROW_GROUP_SIZE_BYTES,
"Unknown option for FastLanes"); here it is registered and driven the way
DuckDB's PhysicalCopyToFile drives a CopyFunction (bind, init, sink per chunk,
combine, finalize).  CPU tests: registration and option errors (they fail at
bind, before any scan).  GPU tests: COPY (SELECT ... FROM read_fastlanes(src))
round trips, checked with the oracle on the written file and against the
workload generators."""
import os
import re

import numpy as np
import pytest

from ext_harness import Ext, ExtError


@pytest.fixture(scope="module")
def ext(_built):
    e = Ext()
    yield e
    e.close()


@pytest.fixture
def li_file(fl, tmpfile):
    p = tmpfile("li.fls")
    fl.gen_image("lineitem", 0.01).write(p)
    return p


def test_copy_functions_registered(ext):
    assert ext.has_copy_function("fls") and ext.has_copy_function("fastlane")
    assert not ext.has_copy_function("parquet")


@pytest.mark.parametrize("opts,msg", [
    ({"row_group_size": 1000}, "ROW_GROUP_SIZE must be a multiple of 1024"),
    ({"chunk_size": 131072}, "ROW_GROUP_SIZE must be a multiple of 1024"),
    ({"row_group_size": 0}, "ROW_GROUP_SIZE must be a multiple of 1024"),
    ({"row_group_size": 8192, "row_group_size_bytes": 1 << 24}, "mutually exclusive"),
    ({"row_groups_per_file": 0}, "ROW_GROUPS_PER_FILE must be at least 1"),
    ({"compression": "zstd"}, "^Unknown option for FastLanes: COMPRESSION$"),
])
def test_copy_option_errors(ext, li_file, tmpfile, opts, msg):
    with pytest.raises(ExtError, match=msg):
        ext.copy("read_fastlanes", li_file, tmpfile("o.fls"), **opts)


def test_copy_unknown_format(ext, li_file, tmpfile):
    with pytest.raises(ExtError, match="^Catalog Error: Copy Function with name parquet does not exist!$"):
        ext.copy("read_fastlanes", li_file, tmpfile("o.parquet"), fmt="parquet")


@pytest.mark.gpu
@pytest.mark.parametrize("opts,rgsz", [({}, 65536), ({"ROW_GROUP_SIZE": 8192}, 8192),
                                       ({"chunk_size": 1024}, 1024),
                                       ({"row_group_size_bytes": 16 << 20}, 16384)])
def test_copy_roundtrip_lineitem(fl, ext, ref, gpu, li_file, tmpfile, opts, rgsz):
    dst = tmpfile("copy.fls")
    n = ext.copy("read_fastlanes", li_file, dst, fmt="fastlane", **opts)
    assert n == 60175
    src_rows, src_h, _ = ext.scan_count("read_fastlanes", li_file)
    dst_rows, dst_h, _ = ext.scan_count("read_fastlanes", dst)
    assert (dst_rows, dst_h) == (src_rows, src_h)          # same rows, same bytes, same order
    f = ref.RefFile(open(dst, "rb").read())                 # the oracle reads the written file
    assert f.nrows == n and f.f.rowgroup_size == rgsz
    assert f.nrowgroups == -(-n // rgsz) and f.rowgroup_rows(f.nrowgroups - 1) == n - (f.nrowgroups - 1) * rgsz
    for c, dt in ((0, np.int64), (1, np.int32), (10, np.int32)):
        assert np.array_equal(f.decode_column(c, 4).view(dt), fl.gen_values("lineitem", c, 0, n, dt, 0.01))
    codes = fl.gen_values("lineitem", 14, 0, n, np.uint32, 0.01)
    got = f.strings(f.decode_column(14, 4))
    assert all(got[i] == fl.gen_dict_string("lineitem", 14, int(codes[i])).encode() for i in range(0, n, 37))


@pytest.mark.gpu
def test_copy_projected_to_fls(fl, ext, gpu, li_file, tmpfile):
    dst = tmpfile("proj.fls")
    assert ext.copy("read_fastlanes", li_file, dst, proj=[14, 0], row_group_size=4096) == 60175
    names, types, rows = ext.query("read_fastlanes", dst)
    assert names == ["l_shipmode", "l_orderkey"] and types == ["VARCHAR", "BIGINT"]
    okey = fl.gen_values("lineitem", 0, 0, 60175, np.int64, 0.01)
    assert [int(r[1]) for r in rows[::101]] == okey[::101].tolist()
    # replacement scan on the new file, FROM 'proj.fls'
    assert ext.query(None, dst, limit=3)[2] == rows[:3]


@pytest.mark.parametrize("threads", [1, 3])
def test_copy_null_values_round_trip_cpu(ext, ref, tmpfile, threads):
    """COPY of NULL-bearing columns (INTEGER, BIGINT, DOUBLE, VARCHAR; leading,
    sparse, whole-vector and all-NULL stretches, over several row groups and
    sink threads): the file's validity (oracle flsref_validity) marks exactly
    the NULL cells, and every other cell decodes to its value."""
    n = 3 * 4096 + 777
    rng = np.random.default_rng(threads)
    null = rng.random((4, n)) < np.array([[0.1], [0.01], [0.3], [0.2]])
    null[0, :3] = True
    null[2, 4096:5120] = True
    a = [None if null[0, i] else (i * 7919) % 100003 - 50000 for i in range(n)]
    b = [None if null[1, i] else i * 3 for i in range(n)]
    d = [None if null[2, i] else i / 8 for i in range(n)]
    s = [None if null[3, i] else f"s{i % 13}" * (i % 5) for i in range(n)]
    z = [None] * n
    dst = tmpfile(f"nulls{threads}.fls")
    assert ext.copy_values([("a", "INTEGER", a), ("b", "BIGINT", b), ("d", "DOUBLE", d), ("s", "VARCHAR", s),
                            ("z", "BIGINT", z), ("k", "BIGINT", list(range(n)))], dst, threads=threads,
                           row_group_size=4096) == n
    rf = ref.RefFile(open(dst, "rb").read())
    k = np.concatenate([rf.decode(5, g) for g in range(rf.nrowgroups)]).view(np.int64)
    order = np.argsort(k)
    assert np.array_equal(k[order], np.arange(n))
    for c, (vals, dt) in enumerate([(a, np.int32), (b, np.int64), (d, np.float64), (s, None), (z, np.int64)]):
        ok = rf.valid_column(c)[order]
        assert np.array_equal(ok, np.array([v is not None for v in vals])), c
        if dt is None:
            col = rf.strings_column(c)
            got = [col[i] for i in order]
            assert all(got[i] == vals[i].encode() for i in range(n) if ok[i])
        else:
            got = np.concatenate([rf.decode(c, g) for g in range(rf.nrowgroups)]).view(dt)[order]
            assert all(got[i] == vals[i] for i in range(n) if ok[i]), c


def test_copy_values_roundtrip_cpu(ext, ref, tmpfile):
    """The same VALUES source without NULLs writes a file whose oracle decode
    (oracle/flsref.c) returns the values: 5000 rows over two chunks-worth of
    STANDARD_VECTOR_SIZE and a partial vector."""
    n = 5000
    a = [(i * 7919) % 100003 - 50000 for i in range(n)]
    s = [f"s{i % 13}" * (i % 5) for i in range(n)]
    dst = tmpfile("vals.fls")
    assert ext.copy_values([("a", "INTEGER", a), ("s", "VARCHAR", s)], dst) == n
    rf = ref.RefFile(open(dst, "rb").read())
    assert rf.nrows == n
    assert rf.decode(0, 0).view(np.int32).tolist() == a
    assert rf.strings_column(1) == [x.encode() for x in s]


@pytest.mark.parametrize("fail_rg", [0, 1])
def test_copy_background_writer_failure_is_reported(ext, tmpfile, monkeypatch, fail_rg):
    """The COPY sink encodes row group k on a background thread while it
    buffers k+1: a writer failure there must still fail the COPY, with the
    writer's message, whether it hits a full row group (reported at the next
    hand-off or at finalize) or the last, partial one (finalize)."""
    monkeypatch.setenv("FLS_TEST_FAIL_WRITER_RG", str(fail_rg))
    n = 65536 + 1000
    with pytest.raises(ExtError, match="injected writer failure at row group %d" % fail_rg):
        ext.copy_values([("a", "INTEGER", list(range(n)))], tmpfile("fail.fls"))


@pytest.mark.parametrize("batch,pipeline", [("1", "1"), ("2", "1"), ("8", "1"), ("1", "0"), ("2", "0")])
def test_copy_batches_of_row_groups_cpu(ext, ref, tmpfile, monkeypatch, batch, pipeline):
    """The sink hands the writer FLS_COPY_BATCH row groups per call
    (fls_writer_add_rowgroups): 4 row groups, the last partial, in batches of
    1, 2 and 8 decode (oracle) to the source values, VARCHAR offsets included;
    with the writer calls pipelined (fls_writer_set_pipelined, the default) or
    not (FLS_COPY_PIPELINE=0) -- the same file."""
    monkeypatch.setenv("FLS_COPY_BATCH", batch)
    monkeypatch.setenv("FLS_COPY_PIPELINE", pipeline)
    n = 3 * 65536 + 1000
    a = [(i * 7919) % 100003 - 50000 for i in range(n)]
    s = [f"w{i % 7}" * (i % 11) for i in range(n)]  # 0..20 bytes: inlined and pointer string_t
    dst = tmpfile(f"batch{batch}_{pipeline}.fls")
    assert ext.copy_values([("a", "INTEGER", a), ("s", "VARCHAR", s)], dst) == n
    if batch == "2":
        # the same bytes either way
        other = tmpfile(f"batch{batch}_{pipeline}_other.fls")
        monkeypatch.setenv("FLS_COPY_PIPELINE", "0" if pipeline == "1" else "1")
        assert ext.copy_values([("a", "INTEGER", a), ("s", "VARCHAR", s)], other) == n
        assert open(other, "rb").read() == open(dst, "rb").read()
    rf = ref.RefFile(open(dst, "rb").read())
    assert rf.nrows == n and rf.nrowgroups == 4
    assert np.concatenate([rf.decode(0, g) for g in range(4)]).view(np.int32).tolist() == a
    assert rf.strings_column(1) == [x.encode() for x in s]


def test_copy_lone_sink_column_helpers_same_bytes(ext, tmpfile, monkeypatch):
    """A lone sink (an ordered COPY's) copies each slice's columns on helper
    threads (FLS_COPY_SINK_THREADS, default 4): the file is the one the sink
    writes alone, NULLs, inlined and pointer strings and a partial row group
    included."""
    n = 2 * 65536 + 3000
    a = [None if i % 97 == 0 else (i * 7919) % 100003 - 50000 for i in range(n)]
    s = [None if i % 89 == 0 else f"w{i % 7}" * (i % 11) for i in range(n)]
    d = [i / 4 for i in range(n)]
    cols = [("a", "INTEGER", a), ("s", "VARCHAR", s), ("d", "DOUBLE", d), ("t", "VARCHAR", [f"x{i % 3}" for i in range(n)])]
    out = {}
    for th in ("0", "4"):
        monkeypatch.setenv("FLS_COPY_SINK_THREADS", th)
        dst = tmpfile(f"helpers{th}.fls")
        assert ext.copy_values(cols, dst) == n
        out[th] = open(dst, "rb").read()
    assert out["0"] == out["4"]


@pytest.mark.parametrize("fmt", ["fls", "fastlane"])
def test_copy_execution_mode_and_batch_size(ext, fmt):
    """Like the reference's registration (src/writer/write_fastlane_stream.cpp:
    251-265): an unordered COPY runs parallel sinks, the desired batch is one
    row group (ROW_GROUP_SIZE); an ordered COPY keeps one sink (REGULAR), also
    for a batch-index source, since no prepare_batch / flush_batch exist."""
    assert ext.copy_mode(fmt, preserve=False, batch_index=False) == (1, 65536)
    assert ext.copy_mode(fmt, preserve=False, batch_index=True) == (1, 65536)
    assert ext.copy_mode(fmt, preserve=True, batch_index=False)[0] == 0
    assert ext.copy_mode(fmt, preserve=True, batch_index=True)[0] == 0
    assert ext.copy_mode(fmt, True, True, {"ROW_GROUP_SIZE": 8192}) == (0, 8192)


@pytest.mark.parametrize("threads,batch", [(1, "8"), (4, "8"), (4, "1"), (3, "3")])
def test_copy_parallel_sinks_cpu(ext, ref, tmpfile, monkeypatch, threads, batch):
    """An unordered COPY (PARALLEL_COPY_TO_FILE) runs a sink per thread, each
    into its own stage; full batches of row groups go to the writer from the
    stages and the remainders merge at combine.  The file holds every source
    row exactly once (order unpromised, so compared as a multiset of (a, s)
    pairs), every row group but the last is full, and with one thread the
    row order is the input's."""
    monkeypatch.setenv("FLS_COPY_BATCH", batch)
    rg = 1024
    n = 37 * rg + 517
    a = [(i * 7919) % 100003 - 50000 for i in range(n)]
    s = [f"p{i % 7}" * (i % 11) for i in range(n)]  # inlined and pointer string_t
    dst = tmpfile(f"par{threads}_{batch}.fls")
    assert ext.copy_values([("a", "INTEGER", a), ("s", "VARCHAR", s)], dst, threads=threads,
                           row_group_size=rg) == n
    rf = ref.RefFile(open(dst, "rb").read())
    assert rf.nrows == n and rf.f.rowgroup_size == rg and rf.nrowgroups == -(-n // rg)
    assert all(rf.rowgroup_rows(g) == rg for g in range(rf.nrowgroups - 1))
    got_a = np.concatenate([rf.decode(0, g) for g in range(rf.nrowgroups)]).view(np.int32).tolist()
    got_s = rf.strings_column(1)
    if threads == 1:
        assert got_a == a and got_s == [x.encode() for x in s]
    assert sorted(zip(got_a, got_s)) == sorted(zip(a, (x.encode() for x in s)))


@pytest.mark.parametrize("budget_mb", [None, "1"])
def test_copy_many_sinks_bounded_staging_cpu(ext, ref, tmpfile, monkeypatch, capfd, budget_mb):
    """36 sink threads each buffering up to FLS_COPY_BATCH = 8 row groups
    would stage ~9 MB here; past FLS_COPY_STAGED_MB (all stages together) a
    stage hands its rows over at its next row-group boundary, so the peak
    stays within the budget plus one row group per stage.  Every row arrives
    exactly once either way."""
    monkeypatch.setenv("FLS_COPY_PROFILE", "1")
    if budget_mb:
        monkeypatch.setenv("FLS_COPY_STAGED_MB", budget_mb)
    else:
        monkeypatch.delenv("FLS_COPY_STAGED_MB", raising=False)
    rg, threads = 1024, 36
    n = threads * 8 * rg + 77
    a = [(i * 104729) % 1000003 for i in range(n)]
    s = [f"q{i % 13}" * (i % 9) for i in range(n)]  # 0..27 bytes: inlined and arena strings
    dst = tmpfile(f"many_{budget_mb}.fls")
    capfd.readouterr()
    assert ext.copy_values([("a", "BIGINT", a), ("s", "VARCHAR", s)], dst, threads=threads,
                           row_group_size=rg) == n
    err = capfd.readouterr().err
    m = re.search(r"peak staged (\d+) bytes", err)
    assert m, err
    peak = int(m.group(1))
    rg_bytes = rg * (8 + 16) + max(sum(len(x) for x in s[k:k + rg] if len(x) > 12) for k in range(0, n, rg))
    if budget_mb:
        assert peak <= (int(budget_mb) << 20) + threads * rg_bytes
    rf = ref.RefFile(open(dst, "rb").read())
    assert rf.nrows == n
    got_a = np.concatenate([rf.decode(0, g) for g in range(rf.nrowgroups)]).view(np.int64).tolist()
    assert sorted(zip(got_a, rf.strings_column(1))) == sorted(zip(a, (x.encode() for x in s)))


@pytest.mark.parametrize("threads", [1, 3])
def test_copy_row_groups_per_file_rotates_cpu(ext, ref, tmpfile, threads):
    """ROW_GROUPS_PER_FILE (reference write_fastlane_stream.cpp:96-97,
    :267-289): the COPY target becomes a directory of data_<i>.fls files, and
    DuckDB opens the next file once the current one holds that many row
    groups (asked before each sink, so a file can end past the boundary by
    the chunks in flight).  Every row lands in exactly one file; one sink
    thread keeps the order and fills every file but the last with exactly
    ROW_GROUPS_PER_FILE row groups."""
    rg, per = 1024, 2
    n = 5 * rg + 300
    a = [(i * 37) % 1009 for i in range(n)]
    s = [f"r{i % 9}" * (i % 6) for i in range(n)]
    d = tmpfile(f"rot{threads}")
    assert ext.copy_values([("a", "BIGINT", a), ("s", "VARCHAR", s)], d, threads=threads,
                           row_group_size=rg, row_groups_per_file=per) == n
    files = sorted(os.listdir(d), key=lambda f: int(f[5:-4]))
    assert files == [f"data_{i}.fls" for i in range(len(files))]
    got, sizes = [], []
    for f in files:
        rf = ref.RefFile(open(os.path.join(d, f), "rb").read())
        sizes.append(rf.nrows)
        assert rf.f.rowgroup_size == rg
        va = np.concatenate([rf.decode(0, g) for g in range(rf.nrowgroups)]).view(np.int64).tolist()
        got += list(zip(va, rf.strings_column(1)))
    exp = list(zip(a, (x.encode() for x in s)))
    if threads == 1:
        assert sizes == [per * rg, per * rg, n - 2 * per * rg] and got == exp
    else:
        assert min(sizes) > 0 and max(sizes) <= per * rg + threads * 2048
    assert sorted(got) == sorted(exp)


@pytest.mark.gpu
def test_copy_rotated_files_read_back_with_glob(ext, gpu, tmpfile):
    """read_fastlanes('dir/*.fls') over a rotated COPY's files returns every
    row once (the multi-file scan reads them as one table)."""
    rg = 1024
    n = 7 * rg + 5
    d = tmpfile("rotg")
    assert ext.copy_values([("a", "BIGINT", list(range(n)))], d, threads=2, row_group_size=rg,
                           row_groups_per_file=3) == n
    assert len(os.listdir(d)) >= 2
    names, types, rows = ext.query("read_fastlanes", os.path.join(d, "*.fls"), threads=2)
    assert types == ["BIGINT"] and sorted(int(r[0]) for r in rows) == list(range(n))


@pytest.mark.gpu
def test_copy_parallel_from_scan(fl, ext, ref, gpu, li_file, tmpfile):
    """COPY (SELECT * FROM read_fastlanes(src)) TO dst with a parallel scan and
    four sink threads: every row once (multiset of (l_orderkey, l_partkey,
    l_shipmode code) triples vs the generator), only the last row group short."""
    dst = tmpfile("par.fls")
    n = ext.copy("read_fastlanes", li_file, dst, threads=4, row_group_size=4096)
    assert n == 60175
    f = ref.RefFile(open(dst, "rb").read())
    assert f.nrows == n and f.nrowgroups == -(-n // 4096)
    assert all(f.rowgroup_rows(g) == 4096 for g in range(f.nrowgroups - 1))
    k0 = f.decode_column(0, 4).view(np.int64)
    k1 = f.decode_column(1, 4).view(np.int32)
    s14 = f.strings(f.decode_column(14, 4))
    e0 = fl.gen_values("lineitem", 0, 0, n, np.int64, 0.01)
    e1 = fl.gen_values("lineitem", 1, 0, n, np.int32, 0.01)
    codes = fl.gen_values("lineitem", 14, 0, n, np.uint32, 0.01)
    modes = {int(c): fl.gen_dict_string("lineitem", 14, int(c)).encode() for c in np.unique(codes)}
    got = sorted(zip(k0.tolist(), k1.tolist(), s14))
    want = sorted(zip(e0.tolist(), e1.tolist(), (modes[int(c)] for c in codes)))
    assert got == want


def test_copy_string_limit_is_per_row_group_cpu(tmpfile):
    """The writer's string offsets are 32-bit per row group (the sink restarts
    them at every row group of a batch): with the limit lowered to 100 KB by
    a test hook, a batch of row groups holding 60 KB of strings each is
    written, and a row group holding 150 KB fails with the per-row-group
    message.  (Run in a child process: the hook is read once.)"""
    import subprocess
    import sys
    code = f"""
import sys; sys.path.insert(0, 'tests')
from ext_harness import Ext, ExtError
e = Ext()
rg = 1024
ok = [("x" * 60) for _ in range(4 * rg)]            # 60 KB per row group, 240 KB per batch
assert e.copy_values([("s", "VARCHAR", ok)], {tmpfile('ok.fls')!r}, row_group_size=rg) == len(ok)
big = [("y" * 150) for _ in range(rg)]               # 150 KB in one row group
try:
    e.copy_values([("s", "VARCHAR", big)], {tmpfile('big.fls')!r}, row_group_size=rg)
    print("no error")
except ExtError as x:
    print(str(x))
"""
    root = str(__import__("pathlib").Path(__file__).parents[1])
    out = subprocess.run([sys.executable, "-c", code], env={**os.environ, "FLS_TEST_STRING_LIMIT": "100000"},
                         capture_output=True, text=True, timeout=120, cwd=root)
    assert out.returncode == 0, out.stderr
    assert 'column "s" holds more than 4 GiB of strings in one row group' in out.stdout, out.stdout
