"""CPU writer (the .fls producer, reference write path stubs
src/writer/write_fastlane*.cpp) round-trips through the oracle, for every
encoding, type and the seeded workloads."""
import ctypes

import numpy as np
import pytest

from helpers import INT_TYPE, SIGNED, width_sweep_values


def roundtrip(fl, ref, cols):
    img = fl.write_image(cols)
    rf = ref.RefFile(img)
    for c, spec in enumerate(cols):
        ty, vals = spec[1], spec[2]
        raw = np.concatenate([rf.decode(c, rg) for rg in range(rf.nrowgroups)])
        if ty == fl.VARCHAR:
            assert rf.strings(raw) == [v.encode() for v in vals]
        else:
            assert np.array_equal(raw.view(fl.NP_DTYPE[ty]), np.asarray(vals).astype(fl.NP_DTYPE[ty]))
    return img, rf


@pytest.mark.parametrize("enc", [1, 2, 3, 4, 0])
@pytest.mark.parametrize("T", [8, 16, 32, 64])
def test_int_roundtrip(fl, ref, enc, T):
    rng = np.random.default_rng(T * 10 + enc)
    if enc == 3:  # dictionary: bounded cardinality
        v = rng.integers(-100, 100, 5000).astype(SIGNED[T])
    elif enc == 4:
        v = np.repeat(rng.integers(-100, 100, 100), 50).astype(SIGNED[T])
    else:
        v = width_sweep_values(T, rng)
    roundtrip(fl, ref, [("v", INT_TYPE[T], v, enc)])


def test_unsigned_date_decimal(fl, ref):
    rng = np.random.default_rng(1)
    n = 70001
    roundtrip(fl, ref, [("u8", fl.UINT8, rng.integers(0, 256, n), fl.ENC_AUTO),
                        ("u64", fl.UINT64, rng.integers(0, 2**63, n, dtype=np.uint64) * np.uint64(2), fl.ENC_FFOR),
                        ("d", fl.DATE, 8035 + rng.integers(0, 2557, n), fl.ENC_AUTO),
                        ("m", fl.DECIMAL, rng.integers(-10**12, 10**12, n), fl.ENC_AUTO, 15, 2)])


def test_strings(fl, ref):
    rng = np.random.default_rng(2)
    words = ["", "x", "ümlaut ✓", "a" * 300] + [f"s{i}" for i in range(3000)]
    v = [words[i] for i in rng.integers(0, len(words), 140000)]
    roundtrip(fl, ref, [("s", fl.VARCHAR, v, fl.ENC_DICT)])


def test_auto_picks_compact_encodings(fl, ref):
    n = 65536
    cols = [("sorted", fl.INT64, np.arange(n) * 3 + 10**15, fl.ENC_AUTO),
            ("runs", fl.INT32, np.repeat(np.random.default_rng(0).integers(-2**31, 2**31 - 1, n // 1000 + 1),
                                         1000)[:n], fl.ENC_AUTO),
            ("few", fl.INT64, (np.arange(n) % 3) * 10**17, fl.ENC_AUTO)]
    img, rf = roundtrip(fl, ref, cols)
    import struct
    raw = img.tobytes()
    encs = []
    for c in range(3):
        # chunk header encoding byte (offset 4) of row group 0
        foff = struct.unpack_from("<Q", raw, len(raw) - 16)[0]
        p = foff + 32
        for _ in range(rf.ncols):
            p += 6 + struct.unpack_from("<H", raw, p + 4)[0]
        off = struct.unpack_from("<Q", raw, p + 4 + 16 * c)[0]
        encs.append(raw[off + 4])
    assert encs[0] == 2          # DELTA for a sorted run of keys
    assert encs[1] in (3, 4)     # DICT or RLE for long runs
    assert encs[2] == 3          # DICT for 3 distinct 64-bit values
    assert img.len < n * 3       # well under one byte per value overall


def test_writer_errors(fl):
    with pytest.raises(fl.FlsError, match="VARCHAR/BLOB support DICT and FSST"):
        fl.write_image([("s", fl.VARCHAR, ["a"], fl.ENC_FFOR)])
    with pytest.raises(fl.FlsError, match="FLOAT/DOUBLE support ALP"):
        fl.write_image([("d", fl.DOUBLE, [1.5], fl.ENC_FFOR)])
    with pytest.raises(fl.FlsError, match="ALP needs FLOAT/DOUBLE"):
        fl.write_image([("i", fl.INT32, [1], fl.ENC_ALP)])
    with pytest.raises(fl.FlsError, match="FSST needs VARCHAR/BLOB"):
        fl.write_image([("i", fl.INT64, [1], fl.ENC_FSST)])
    with pytest.raises(fl.FlsError, match="unsupported type"):
        fl.write_image([("x", 99, [1], fl.ENC_FFOR)])
    with pytest.raises(ValueError):
        fl.write_image([("a", fl.INT32, [1, 2], fl.ENC_FFOR), ("b", fl.INT32, [1], fl.ENC_FFOR)])


@pytest.mark.parametrize("wl,scale,n", [("c1", 1, 0), ("c3", 1, 300000), ("c4", 1, 200000), ("lineitem", 0.01, 0)])
def test_workloads_match_generator(fl, ref, wl, scale, n):
    img = fl.gen_image(wl, scale, n)
    rf = ref.RefFile(img)
    for c in range(rf.ncols):
        name, ty, _, _ = rf.column(c)
        raw = rf.decode_column(c, 4)
        if ty == fl.VARCHAR:
            codes = fl.gen_values(wl, c, 0, rf.nrows, np.uint32, scale, n)
            d = [fl.gen_dict_string(wl, c, k) for k in range(int(codes.max()) + 1)]
            assert rf.strings(raw) == [d[k].encode() for k in codes], name
        else:
            assert np.array_equal(raw.view(fl.NP_DTYPE[ty]), fl.gen_values(wl, c, 0, rf.nrows, fl.NP_DTYPE[ty], scale, n)), name


def test_lineitem_distributions(fl):
    n = 60175
    g = {c: fl.gen_values("lineitem", c, 0, n, t, 0.01) for c, t in
         [(0, np.int64), (3, np.int32), (4, np.int64), (6, np.int64), (10, np.int32), (12, np.int32)]}
    assert np.all(np.diff(g[0]) >= 0)                       # orderkey sorted
    assert g[3].min() == 1 and g[3].max() == 7              # 1..7 lines per order
    assert g[4].min() == 100 and g[4].max() == 5000         # quantity 1..50 (cents)
    assert g[6].min() == 0 and g[6].max() == 10             # discount 0.00..0.10
    assert g[10].min() >= 8036 and g[12].max() <= 10591 + 151
    # keys dense 8 per 32
    assert set((np.unique(g[0]) - 1) % 32) <= set(range(8))
    assert fl.gen_nrows("lineitem", 100) == 600037902 and fl.gen_nrows("lineitem", 1) == 6001215


def test_shard_images_concatenate(fl, ref):
    """Row-group shards (what each rank encodes) reassemble the full table."""
    full = ref.RefFile(fl.gen_image("c3", nrows=7 * 65536 + 123))
    parts = [fl.gen_image("c3", nrows=7 * 65536 + 123, rg_begin=b, rg_end=e) for b, e in [(0, 3), (3, 5), (5, 8)]]
    got = np.concatenate([ref.RefFile(p).decode_column(0) for p in parts])
    assert np.array_equal(got, full.decode_column(0))
    assert [ref.RefFile(p).f.row_offset for p in parts] == [0, 3 * 65536, 5 * 65536]


@pytest.mark.parametrize("rgsz", [1024, 4096, 20480])
def test_custom_rowgroup_size(fl, ref, rgsz):
    # COPY ... (ROW_GROUP_SIZE n) -- src/writer/write_fastlane_stream.cpp:75-90
    rng = np.random.default_rng(rgsz)
    n = 3 * rgsz + 555
    a = rng.integers(-1000, 1000, n).astype(np.int32)
    s = [f"k{i % 13}" for i in range(n)]
    img = fl.write_image([("a", fl.INT32, a, fl.ENC_AUTO), ("s", fl.VARCHAR, s, fl.ENC_DICT)], rowgroup=rgsz)
    rf = ref.RefFile(img)
    assert rf.f.rowgroup_size == rgsz and rf.nrowgroups == 4
    assert [rf.rowgroup_rows(g) for g in range(4)] == [rgsz] * 3 + [555]
    assert np.array_equal(rf.decode_column(0).view(np.int32), a)
    assert rf.strings(rf.decode_column(1)) == [x.encode() for x in s]


@pytest.mark.parametrize("rgsz", [0, 1000, 65537, 131072])
def test_bad_rowgroup_size_rejected(fl, rgsz):
    with pytest.raises(fl.FlsError):
        fl.write_image([("a", fl.INT32, np.arange(10), fl.ENC_FFOR)], rowgroup=rgsz)


def _empty_image(fl):
    return fl.write_image([("a", fl.INT32, np.zeros(0, np.int32), fl.ENC_FFOR),
                           ("s", fl.VARCHAR, [], fl.ENC_AUTO)])


def test_empty_table_scans_nothing_without_a_gpu(fl, ref):
    """A table with columns but no rows: schema, no row groups, and a scan
    that ends at once (no device work, so this runs without a GPU)."""
    img = _empty_image(fl)
    rf = ref.RefFile(img)
    assert rf.nrows == 0 and rf.nrowgroups == 0
    t = fl.Connection().read_image(img)
    assert (t.nrows, t.nrowgroups, t.ncols) == (0, 0, 2)
    assert [c[0] for c in t.schema()] == ["a", "s"]
    assert list(t.scan()) == []
    # an empty row-group range of a non-empty table is empty too
    t2 = fl.Connection().read_image(fl.write_image([("a", fl.INT32, np.arange(10, dtype=np.int32), fl.ENC_FFOR)]))
    assert list(t2.scan(rg_begin=1, rg_end=1)) == []


def test_filter_pruning_everything_scans_nothing(fl):
    """Zone maps prune every row group: the scan ends without device work."""
    img = fl.write_image([("k", fl.INT64, np.arange(200000, dtype=np.int64), fl.ENC_DELTA)])
    t = fl.Connection().read_image(img)
    assert list(t.scan_filtered([(0, ">", 10 ** 9)])) == []
    assert t.pruned == t.nrowgroups


@pytest.mark.gpu
def test_gpu_empty_table_device_paths(fl, gpu):
    t = fl.Connection().read_image(_empty_image(fl))
    assert list(t.scan()) == []
    with pytest.raises(fl.FlsError, match="out of bounds"):
        t.device_upload()


def _mixed_columns(fl, n, seed):
    rng = np.random.default_rng(seed)
    words = ["alpha", "beta", "gamma", "a much longer string value %d" % seed, ""]
    return [("k", fl.INT64, np.cumsum(rng.integers(0, 5, n)), fl.ENC_AUTO),
            ("q", fl.INT32, rng.integers(1, 51, n), fl.ENC_AUTO),
            ("r", fl.INT16, np.repeat(rng.integers(-9, 9, n // 50 + 1), 50)[:n], fl.ENC_AUTO),
            ("d", fl.DOUBLE, np.round(rng.random(n) * 1000, 2), fl.ENC_AUTO),
            ("s", fl.VARCHAR, [words[i] for i in rng.integers(0, len(words), n)], fl.ENC_AUTO),
            ("t", fl.VARCHAR, ["comment %d of row %d" % (x, i) for i, x in enumerate(rng.integers(0, 10**6, n))],
             fl.ENC_FSST)]


@pytest.mark.parametrize("batch,threads,rgsz,n", [(8, 8, 1024, 9 * 1024 + 17), (3, 4, 2048, 7 * 2048),
                                                   (16, 1, 1024, 5000), (4, 8, 65536, 65536 * 2 + 5)])
def test_add_rowgroups_batches_match_single_calls(fl, ref, batch, threads, rgsz, n):
    # fls_writer_add_rowgroups: (row group, column) tasks across the batch,
    # the same file as one fls_writer_add_rowgroup call per row group
    cols = _mixed_columns(fl, n, batch + rgsz)
    one = fl.write_image(cols, rowgroup=rgsz, threads=1)
    many = fl.write_image(cols, rowgroup=rgsz, batch=batch, threads=threads)
    assert bytes(one.view()) == bytes(many.view())
    rf = ref.RefFile(many)
    assert rf.nrows == n and rf.nrowgroups == (n + rgsz - 1) // rgsz


def test_add_rowgroups_rejects_short_group_before_the_last(fl):
    import ctypes as C
    lib = fl.lib
    w = lib.fls_writer_new(0)
    try:
        fl._check(lib.fls_writer_set_rowgroup_size(w, 1024))
        fl._check(lib.fls_writer_add_column(w, b"v", fl.INT32, 0, 0, fl.ENC_FFOR))
        a, b = np.arange(1000, dtype=np.int32), np.arange(1024, dtype=np.int32)
        rows = (C.c_uint32 * 2)(1000, 1024)
        data = (C.c_void_p * 2)(a.ctypes.data, b.ctypes.data)
        assert lib.fls_writer_add_rowgroups(w, 2, rows, data, None) != 0
        assert "short" in fl.last_error()
        rows = (C.c_uint32 * 2)(1024, 1000)
        data = (C.c_void_p * 2)(b.ctypes.data, a.ctypes.data)
        fl._check(lib.fls_writer_add_rowgroups(w, 2, rows, data, None))
        # nothing may follow a short row group
        assert lib.fls_writer_add_rowgroups(w, 1, (C.c_uint32 * 1)(1024), (C.c_void_p * 1)(b.ctypes.data), None) != 0
    finally:
        lib.fls_writer_free(w)


@pytest.mark.parametrize("threads", [1, 8])
def test_finish_file_writes_the_image_bytes(fl, tmp_path, threads):
    # fls_writer_finish_file pwrite()s every chunk at its offset from the
    # writer's threads (no whole-file image): the same bytes as
    # fls_writer_finish_image, NULL-bearing chunks (validity appended) included
    n = 5 * 1024 + 300
    cols = _mixed_columns(fl, n, 7)
    rng = np.random.default_rng(3)
    cols.append(("nv", fl.INT32, np.ma.masked_array(rng.integers(0, 100, n), mask=rng.random(n) < 0.1),
                 fl.ENC_AUTO))
    cols.append(("ns", fl.VARCHAR, [None if i % 7 == 0 else "v%d" % (i % 13) for i in range(n)], fl.ENC_AUTO))
    img = fl.write_image(cols, rowgroup=1024, batch=4, threads=threads)
    path = tmp_path / "t.fls"
    assert fl.write_image(cols, rowgroup=1024, batch=4, threads=threads, path=path) is None
    assert path.read_bytes() == bytes(img.view())


@pytest.mark.parametrize("batch", [1, 3, 8])
def test_streamed_output_writes_the_image_bytes(fl, tmp_path, batch):
    # fls_writer_set_output: complete row groups stream to a temporary file
    # beside the path while later ones encode, the footer is added and the
    # file renamed over the path at finish -- the same bytes as the image
    n = 9 * 1024 + 77
    cols = _mixed_columns(fl, n, 11)
    rng = np.random.default_rng(5)
    cols.append(("nv", fl.INT64, np.ma.masked_array(rng.integers(-9, 9, n), mask=rng.random(n) < 0.2),
                 fl.ENC_AUTO))
    cols.append(("ns", fl.VARCHAR, [None if i % 5 == 0 else "s%d" % (i % 31) for i in range(n)], fl.ENC_FSST))
    img = fl.write_image(cols, rowgroup=1024, batch=batch, threads=4)
    path = tmp_path / "s.fls"
    path.write_bytes(b"old contents")  # replaced whole, never partly overwritten
    assert fl.write_image(cols, rowgroup=1024, batch=batch, threads=4, path=path, stream=True) is None
    assert path.read_bytes() == bytes(img.view())
    assert sorted(p.name for p in tmp_path.iterdir()) == ["s.fls"]   # no temporary file left


@pytest.mark.parametrize("batch,stream", [(1, False), (3, True), (8, True)])
def test_pipelined_adds_write_the_same_bytes(fl, tmp_path, batch, stream):
    # fls_writer_set_pipelined: a call returns with its chunk tasks queued
    # behind the previous call's; row groups still go in in call order
    n = 13 * 1024 + 5
    cols = _mixed_columns(fl, n, 17)
    cols.append(("ns", fl.VARCHAR, [None if i % 3 == 0 else "p%d" % (i % 23) for i in range(n)], fl.ENC_FSST))
    img = fl.write_image(cols, rowgroup=1024, batch=batch, threads=4)
    piped = fl.write_image(cols, rowgroup=1024, batch=batch, threads=4, pipelined=True)
    assert bytes(piped.view()) == bytes(img.view())
    path = tmp_path / "p.fls"
    assert fl.write_image(cols, rowgroup=1024, batch=batch, threads=4, path=path, stream=stream,
                          pipelined=True) is None
    assert path.read_bytes() == bytes(img.view())


def test_pipelined_short_row_group_rule_sees_the_pending_call(fl):
    # the previous call's row groups are still encoding, but a short one
    # among them still ends the file
    w = fl.lib.fls_writer_new(0)
    try:
        assert fl.lib.fls_writer_set_rowgroup_size(w, 1024) == 0
        assert fl.lib.fls_writer_add_column(w, b"x", fl.INT32, 0, 0, fl.ENC_FFOR) == 0
        assert fl.lib.fls_writer_set_pipelined(w, 1) == 0
        x = np.arange(1024, dtype=np.int32)
        data = (ctypes.c_void_p * 1)(x.ctypes.data)
        assert fl.lib.fls_writer_add_rowgroup(w, 1000, data, None) == 0
        assert fl.lib.fls_writer_add_rowgroup(w, 1024, data, None) < 0
        assert "only the last row group" in fl.last_error()
        # the failed call settled the pending one: its buffers are free now
        x[:] = -1
        assert fl.lib.fls_writer_set_rowgroup_size(w, 2048) < 0   # a row group is pending
        assert fl.lib.fls_writer_set_pipelined(w, 0) == 0
        p, ln = ctypes.c_void_p(), ctypes.c_uint64()
        assert fl.lib.fls_writer_finish_image(w, ctypes.byref(p), ctypes.byref(ln)) == 0
        img = ctypes.string_at(p, ln.value)
        fl.lib.fls_image_free(p)
    finally:
        fl.lib.fls_writer_free(w)
    # the one row group holds 0..999 (written before x was overwritten)
    ref = fl.write_image([("x", fl.INT32, np.arange(1000, dtype=np.int32), fl.ENC_FFOR)], rowgroup=1024)
    assert img == bytes(ref.view())


def test_pipelined_free_without_finish_waits_for_pending(fl):
    # freeing a pipelined writer whose last call is still encoding waits for
    # it (its tasks read the caller's buffers) -- no crash, nothing leaks
    for _ in range(3):
        w = fl.lib.fls_writer_new(0)
        try:
            assert fl.lib.fls_writer_set_rowgroup_size(w, 1024) == 0
            assert fl.lib.fls_writer_add_column(w, b"s", fl.VARCHAR, 0, 0, fl.ENC_AUTO) == 0
            assert fl.lib.fls_writer_set_threads(w, 4) == 0
            assert fl.lib.fls_writer_set_pipelined(w, 1) == 0
            strs = [b"pending row %d" % i for i in range(8 * 1024)]
            buf = np.frombuffer(b"".join(strs), dtype=np.uint8).copy()
            offs = np.zeros(len(strs) + 1, dtype=np.uint32)
            offs[1:] = np.cumsum([len(x) for x in strs])
            nrows = (ctypes.c_uint32 * 8)(*([1024] * 8))
            data = (ctypes.c_void_p * 8)(*[buf.ctypes.data] * 8)
            op = (ctypes.c_void_p * 8)(*[offs.ctypes.data + 4 * 1024 * k for k in range(8)])
            # row group k: strings [1024 k, 1024 k + 1024), offsets relative to buf
            assert fl.lib.fls_writer_add_rowgroups(w, 8, nrows, data, op) == 0
        finally:
            fl.lib.fls_writer_free(w)


def test_pipelined_image_matches_across_thread_counts(fl):
    # any thread count, pipelined, writes the unpipelined image's bytes
    n = 9 * 1024 + 11
    cols = _mixed_columns(fl, n, 23)
    ref = fl.write_image(cols, rowgroup=1024, batch=2, threads=3).tobytes()
    for threads in (1, 2, 7):
        got = fl.write_image(cols, rowgroup=1024, batch=2, threads=threads, pipelined=True).tobytes()
        assert got == ref


def test_streamed_output_abandoned_leaves_nothing(fl, tmp_path):
    # a writer freed without its finish (a failed COPY) removes its temporary
    # file and leaves the destination as it was
    path = tmp_path / "a.fls"
    path.write_bytes(b"keep me")
    w = fl.lib.fls_writer_new(0)
    try:
        assert fl.lib.fls_writer_add_column(w, b"x", fl.INT32, 0, 0, fl.ENC_FFOR) == 0
        assert fl.lib.fls_writer_set_output(w, str(path).encode()) == 0
        x = np.arange(3000, dtype=np.int32)
        data = (ctypes.c_void_p * 1)(x.ctypes.data)
        assert fl.lib.fls_writer_add_rowgroup(w, 3000, data, None) == 0
        assert len(list(tmp_path.iterdir())) == 2   # the destination + the temporary file
        # another path at finish is refused (and the temporary file removed)
        assert fl.lib.fls_writer_finish_file(w, str(tmp_path / "b.fls").encode()) < 0
    finally:
        fl.lib.fls_writer_free(w)
    assert sorted(p.name for p in tmp_path.iterdir()) == ["a.fls"] and path.read_bytes() == b"keep me"


def test_streamed_output_failed_finish_breaks_the_writer(fl, tmp_path):
    # row groups handed to the stream gave their chunk bytes away;
    # after a failed finish (wrong path) a retry must not build a file or an
    # image from the emptied chunks under a valid footer
    path = tmp_path / "r.fls"
    w = fl.lib.fls_writer_new(0)
    try:
        assert fl.lib.fls_writer_set_rowgroup_size(w, 1024) == 0
        assert fl.lib.fls_writer_add_column(w, b"x", fl.INT32, 0, 0, fl.ENC_FFOR) == 0
        assert fl.lib.fls_writer_set_output(w, str(path).encode()) == 0
        x = np.arange(1024, dtype=np.int32)
        data = (ctypes.c_void_p * 1)(x.ctypes.data)
        for _ in range(3):
            assert fl.lib.fls_writer_add_rowgroup(w, 1024, data, None) == 0
        assert fl.lib.fls_writer_finish_file(w, str(tmp_path / "other.fls").encode()) < 0
        assert fl.lib.fls_writer_finish_file(w, str(path).encode()) < 0
        assert "failed earlier" in fl.last_error()
        p, ln = ctypes.c_void_p(), ctypes.c_uint64()
        assert fl.lib.fls_writer_finish_image(w, ctypes.byref(p), ctypes.byref(ln)) < 0
    finally:
        fl.lib.fls_writer_free(w)
    assert list(tmp_path.iterdir()) == []


def test_streamed_output_wrong_path_before_any_row_group_can_retry(fl, tmp_path):
    # nothing was handed to the stream yet: the data is intact, and a finish
    # with a path (the stream abandoned) writes the whole file
    path = tmp_path / "ok.fls"
    w = fl.lib.fls_writer_new(0)
    try:
        assert fl.lib.fls_writer_add_column(w, b"x", fl.INT32, 0, 0, fl.ENC_FFOR) == 0
        assert fl.lib.fls_writer_set_output(w, str(path).encode()) == 0
        assert fl.lib.fls_writer_finish_file(w, str(tmp_path / "other.fls").encode()) < 0
        x = np.arange(100, dtype=np.int32)
        data = (ctypes.c_void_p * 1)(x.ctypes.data)
        assert fl.lib.fls_writer_add_rowgroup(w, 100, data, None) == 0
        assert fl.lib.fls_writer_finish_file(w, str(path).encode()) == 0
    finally:
        fl.lib.fls_writer_free(w)
    ref = fl.write_image([("x", fl.INT32, np.arange(100, dtype=np.int32), fl.ENC_FFOR)])
    assert path.read_bytes() == bytes(ref.view())


def test_streamed_output_refuses_unwritable_dir_and_late_set(fl, tmp_path):
    w = fl.lib.fls_writer_new(0)
    try:
        assert fl.lib.fls_writer_add_column(w, b"x", fl.INT32, 0, 0, fl.ENC_FFOR) == 0
        assert fl.lib.fls_writer_set_output(w, str(tmp_path / "nodir" / "x.fls").encode()) < 0
        assert "cannot create" in fl.last_error()
        x = np.arange(100, dtype=np.int32)
        data = (ctypes.c_void_p * 1)(x.ctypes.data)
        assert fl.lib.fls_writer_add_rowgroup(w, 100, data, None) == 0
        assert fl.lib.fls_writer_set_output(w, str(tmp_path / "x.fls").encode()) < 0   # after a row group
    finally:
        fl.lib.fls_writer_free(w)
    assert list(tmp_path.iterdir()) == []


def test_finish_file_reports_unwritable_path(fl, tmp_path):
    cols = _mixed_columns(fl, 2000, 1)
    with pytest.raises(fl.FlsError):
        fl.write_image(cols, rowgroup=1024, path=tmp_path / "missing_dir" / "t.fls")
    assert "cannot create" in fl.last_error()
