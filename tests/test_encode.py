"""GPU chunk encoder (csrc/fls_encode.hip): FFOR / DELTA chunks byte-identical
to the CPU writer's (csrc/fls_writer.cpp enc_ffor / enc_delta), which the
oracle tests pin against the restated FastLanes layout.  The write side of the
scan path: SURVEY.md 8(f) row 1 (COPY ... TO (FORMAT FLS); the reference's
writer is a stub, src/writer/write_fastlane_stream.cpp:65-314)."""
import numpy as np
import pytest

from helpers import fsst_text

INT_TYPES = ["INT8", "INT16", "INT32", "INT64", "UINT8", "UINT16", "UINT32", "UINT64", "DATE", "DECIMAL"]


def _columns(fl, n, rng):
    """Every integer type under FFOR and DELTA, with value shapes that hit
    W = 0 (constant), W = T (full range), negative bases, sorted keys."""
    cols = []
    for tn in INT_TYPES:
        ty = getattr(fl, tn)
        dt = np.dtype(fl.NP_DTYPE[ty])
        info = np.iinfo(dt)
        full = rng.integers(info.min, info.max, n, dtype=dt, endpoint=True)
        small = (rng.integers(-50, 50, n) + (int(info.min) + int(info.max)) // 2).astype(dt)
        const = np.full(n, info.max // 3, dtype=dt)
        keys = np.sort(rng.integers(info.min // 2, info.max // 2, n, dtype=dt))
        for enc in (fl.ENC_FFOR, fl.ENC_DELTA):
            e = "ffor" if enc == fl.ENC_FFOR else "delta"
            cols += [(f"{tn}_{e}_full", ty, full, enc), (f"{tn}_{e}_small", ty, small, enc),
                     (f"{tn}_{e}_const", ty, const, enc), (f"{tn}_{e}_keys", ty, keys, enc)]
    return cols


def test_encode_slot_bytes(fl):
    # header + VecMeta[64] + 128 T bytes per vector (W <= T), DELTA + 128 B
    # bases per vector, rounded up to the 256-byte chunk alignment
    def r256(x):
        return (x + 255) // 256 * 256
    assert fl.encode_slot_bytes(fl.INT64, fl.ENC_FFOR) == r256(64 + 64 * 32 + 64 * 128 * 64)
    assert fl.encode_slot_bytes(fl.INT64, fl.ENC_DELTA) == r256(64 + 64 * 32 + 64 * 128 * 64 + 64 * 128)
    assert fl.encode_slot_bytes(fl.INT8, fl.ENC_FFOR, 1024) % 256 == 0
    assert fl.encode_slot_bytes(fl.FLOAT, fl.ENC_ALP) == 0


def test_set_device_rejects_missing_gpu(fl):
    w = fl.lib.fls_writer_new(0)
    try:
        assert fl.lib.fls_writer_set_device(w, 1 << 20) < 0
        assert fl.lib.fls_writer_set_device(w, -1) == 0
    finally:
        fl.lib.fls_writer_free(w)


@pytest.mark.gpu
@pytest.mark.parametrize("n,rowgroup", [(65536 * 2 + 777, 65536), (20000, 4096), (1024, 1024), (1, 65536),
                                        (65536 * 3, 65536),
                                        # > 32 row groups: the writer's two buffer sets take turns
                                        # (async submit of batch k while batch k+1 is staged)
                                        (1024 * 70 + 3, 1024), (200000, 1024)])
def test_gpu_writer_bytes_identical(fl, gpu, n, rowgroup):
    cols = _columns(fl, n, np.random.default_rng(n))
    cpu = fl.write_image(cols, rowgroup=rowgroup).tobytes()
    dev = fl.write_image(cols, rowgroup=rowgroup, device=0).tobytes()
    assert len(cpu) == len(dev)
    assert cpu == dev


@pytest.mark.gpu
def test_gpu_writer_mixed_columns_and_decode(fl, ref, gpu):
    """GPU-encoded FFOR / DELTA columns next to CPU-encoded AUTO / DICT /
    VARCHAR ones in one file; the file decodes exactly on the GPU."""
    from helpers import assert_column_equal, gpu_decode_all
    rng = np.random.default_rng(5)
    n = 150000
    keys = np.cumsum(rng.integers(0, 4, n)).astype(np.int64)
    cols = [("k", fl.INT64, keys, fl.ENC_DELTA), ("q", fl.INT32, rng.integers(-9, 9, n), fl.ENC_FFOR),
            ("a", fl.INT32, rng.integers(0, 3, n), fl.ENC_AUTO), ("d", fl.INT16, rng.integers(0, 5, n), fl.ENC_DICT),
            ("s", fl.VARCHAR, [f"v{i % 7}" for i in range(n)], fl.ENC_AUTO)]
    img = fl.write_image(cols, device=0)
    assert img.tobytes() == fl.write_image(cols).tobytes()
    t, st, out = gpu_decode_all(fl, img)
    rf = ref.RefFile(img)
    for c in range(t.ncols):
        assert_column_equal(fl, rf, c, out[c], img.ptr)


@pytest.mark.gpu
@pytest.mark.parametrize("enc", ["FFOR", "DELTA"])
@pytest.mark.parametrize("tn", ["INT64", "INT32", "INT16", "UINT8"])
def test_gpu_encode_device_resident(fl, gpu, enc, tn):
    """fls_encode_device over a column already in HBM: the chunks, laid end to
    end, are the CPU writer's file body for the same single-column table
    (INT64 runs the u64 kernel, the narrower types the u32 one)."""
    rng = np.random.default_rng(11)
    n = 65536 * 5 + 3000
    ty = getattr(fl, tn)
    dt = np.dtype(fl.NP_DTYPE[ty])
    info = np.iinfo(dt)
    if tn == "INT64":
        vals = np.cumsum(rng.integers(0, 26, n)).astype(np.int64) + 1_000_000
    else:
        vals = rng.integers(int(info.min) // 2, int(info.max) // 2, n).astype(dt)
        if enc == "DELTA":
            vals = np.sort(vals)
    e = getattr(fl, "ENC_" + enc)
    cpu = fl.write_image([("k", ty, vals, e)]).tobytes()
    d_in = fl.DeviceBuffer.from_array(vals)
    slot = fl.encode_slot_bytes(ty, e)
    nrg = (n + 65535) // 65536
    d_out = fl.DeviceBuffer(slot * nrg)
    lens, ms = fl.encode_device(0, ty, e, d_in.ptr, n, d_out.ptr)
    assert ms > 0
    body = b"".join(d_out.read(i * slot, lens[i]) for i in range(nrg))
    assert body == cpu[256:256 + len(body)]
    assert sum(lens) == len(body)
    d_in.free()
    d_out.free()


@pytest.mark.gpu
def test_gpu_encode_device_1e8_keys(fl, gpu):
    """At 1e8 rows: GPU-encoded DELTA chunks of config 3's sorted keys equal the
    CPU writer's chunk for the same row group (sampled row groups)."""
    n = 100_000_000
    vals = fl.gen_values("c3", 0, 0, n, np.int64, 1.0, n)
    d_in = fl.DeviceBuffer.from_array(vals)
    slot = fl.encode_slot_bytes(fl.INT64, fl.ENC_DELTA)
    nrg = (n + 65535) // 65536
    d_out = fl.DeviceBuffer(slot * nrg)
    lens, ms = fl.encode_device(0, fl.INT64, fl.ENC_DELTA, d_in.ptr, n, d_out.ptr)
    for rg in sorted({0, 1, nrg // 2, nrg - 1}):
        part = vals[rg * 65536:(rg + 1) * 65536]
        cpu = fl.write_image([("k", fl.INT64, part, fl.ENC_DELTA)]).tobytes()
        assert d_out.read(rg * slot, lens[rg]) == cpu[256:256 + lens[rg]], rg


def _auto_columns(fl, n, rng):
    """ENC_AUTO columns of every integer type with value shapes that make the
    chooser pick each of FFOR (random), DELTA (sorted keys), RLE (runs of 50
    random values) and DICT (few distinct values spread over the whole range)."""
    cols = []
    for tn in INT_TYPES:
        ty = getattr(fl, tn)
        dt = np.dtype(fl.NP_DTYPE[ty])
        info = np.iinfo(dt)
        rand = rng.integers(info.min, info.max, n, dtype=dt, endpoint=True)
        keys = np.sort(rng.integers(info.min // 4, info.max // 4, n, dtype=dt))
        runs = np.repeat(rng.integers(info.min, info.max, n // 50 + 1, dtype=dt, endpoint=True), 50)[:n]
        spread = rng.integers(info.min, info.max, 6, dtype=dt, endpoint=True)[rng.integers(0, 6, n)]
        small = rng.integers(0, 3, n).astype(dt)
        cols += [(f"{tn}_rand", ty, rand, fl.ENC_AUTO), (f"{tn}_keys", ty, keys, fl.ENC_AUTO),
                 (f"{tn}_runs", ty, runs, fl.ENC_AUTO), (f"{tn}_spread", ty, spread, fl.ENC_AUTO),
                 (f"{tn}_small", ty, small, fl.ENC_AUTO)]
    return cols


def _chunk_encodings(img: bytes):
    """{encoding id: count} over the file's chunks (footer walk, fls_format.hpp)"""
    import struct
    foff, flen = struct.unpack_from("<QI", img, len(img) - 16)
    p = foff
    _, nc, _, nrg, _, _ = struct.unpack_from("<IIQIIQ", img, p)
    p += 32
    for _ in range(nc):
        nl = struct.unpack_from("<H", img, p + 4)[0]
        p += 6 + nl
    out = {}
    for _ in range(nrg):
        p += 4
        for _ in range(nc):
            off, _ln = struct.unpack_from("<QQ", img, p)
            p += 16
            e = img[off + 4]
            out[e] = out.get(e, 0) + 1
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("n,rowgroup", [(65536 * 2 + 777, 65536), (20000, 4096), (1024 * 40 + 9, 1024)])
def test_gpu_writer_auto_bytes_identical(fl, gpu, n, rowgroup):
    """ENC_AUTO integer columns chosen and encoded on the GPU (RLE / DICT
    choices encoded by the host from the staged values): the file is the
    CPU writer's, byte for byte, and every one of the four encodings occurs."""
    cols = _auto_columns(fl, n, np.random.default_rng(n + 1))
    cpu = fl.write_image(cols, rowgroup=rowgroup).tobytes()
    dev = fl.write_image(cols, rowgroup=rowgroup, device=0).tobytes()
    assert len(cpu) == len(dev)
    assert cpu == dev
    encs = _chunk_encodings(cpu)
    # (one-vector row groups hold too few values for RLE to beat DICT)
    for e in (fl.ENC_FFOR, fl.ENC_DELTA, fl.ENC_DICT) + ((fl.ENC_RLE,) if rowgroup > 1024 else ()):
        assert encs.get(e, 0) > 0, (e, encs)


def test_auto_columns_choose_every_encoding(fl):
    # CPU side of the test above: the shapes really cover all four choices
    cols = _auto_columns(fl, 20000, np.random.default_rng(20001))
    encs = _chunk_encodings(fl.write_image(cols, rowgroup=4096).tobytes())
    for e in (fl.ENC_FFOR, fl.ENC_DELTA, fl.ENC_RLE, fl.ENC_DICT):
        assert encs.get(e, 0) > 0, (e, encs)


def _rle_columns(fl, n, rng):
    """Explicit ENC_RLE columns of every integer type: long runs, one value,
    a run per value (1,024 runs per vector, the largest aux block) and runs
    of random lengths."""
    cols = []
    for tn in INT_TYPES:
        ty = getattr(fl, tn)
        dt = np.dtype(fl.NP_DTYPE[ty])
        info = np.iinfo(dt)
        long_runs = np.repeat(rng.integers(info.min, info.max, n // 700 + 1, dtype=dt, endpoint=True), 700)[:n]
        const = np.full(n, info.min, dtype=dt)
        every = rng.integers(info.min, info.max, n, dtype=dt, endpoint=True)
        lens = rng.integers(1, 40, n)
        mixed = np.repeat(rng.integers(info.min, info.max, n, dtype=dt, endpoint=True), lens)[:n]
        cols += [(f"{tn}_long", ty, long_runs, fl.ENC_RLE), (f"{tn}_const", ty, const, fl.ENC_RLE),
                 (f"{tn}_every", ty, every, fl.ENC_RLE), (f"{tn}_mixed", ty, mixed, fl.ENC_RLE)]
    return cols


@pytest.mark.gpu
@pytest.mark.parametrize("n,rowgroup", [(65536 * 2 + 777, 65536), (20000, 4096), (1024 * 3 + 1, 1024), (1, 65536)])
def test_gpu_writer_rle_bytes_identical(fl, ref, gpu, n, rowgroup):
    """RLE chunks written by the GPU (encode_rle_kernel) are the CPU writer's
    bytes, and decode to the input under the oracle."""
    cols = _rle_columns(fl, n, np.random.default_rng(n + 7))
    cpu_img = fl.write_image(cols, rowgroup=rowgroup)
    dev = fl.write_image(cols, rowgroup=rowgroup, device=0).tobytes()
    cpu = cpu_img.tobytes()
    assert len(cpu) == len(dev)
    assert cpu == dev
    assert set(_chunk_encodings(cpu)) == {fl.ENC_RLE}
    rf = ref.RefFile(cpu_img)
    for c, (_, ty, vals, _) in enumerate(cols):
        got = np.concatenate([rf.decode(c, r) for r in range(rf.nrowgroups)])
        assert np.array_equal(got.view(vals.dtype), vals), cols[c][0]


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [5, 16, 40])
@pytest.mark.parametrize("n,rowgroup", [(1024 * 70 + 3, 1024), (65536 * 2 + 777, 65536)])
def test_gpu_writer_batched_rowgroups_bytes_identical(fl, gpu, batch, n, rowgroup):
    """fls_writer_add_rowgroups with the GPU encoder: calls whose row groups
    span the encoder's 32-row-group batches (a batch is submitted mid-call,
    once every row group in it is staged) write the CPU writer's bytes."""
    cols = _auto_columns(fl, n, np.random.default_rng(n + batch)) + \
        [("s", fl.VARCHAR, ["row %d" % (i % 977) for i in range(n)], fl.ENC_AUTO)]
    cpu = fl.write_image(cols, rowgroup=rowgroup).tobytes()
    dev = fl.write_image(cols, rowgroup=rowgroup, device=0, batch=batch, threads=8).tobytes()
    assert cpu == dev
    # pipelined calls (fls_writer_set_pipelined): a call's last segment is
    # still staging into the encoder's batch when the next call adds to it
    piped = fl.write_image(cols, rowgroup=rowgroup, device=0, batch=batch, threads=8, pipelined=True).tobytes()
    assert cpu == piped


def _fsst_columns(fl, n, rng):
    """VARCHAR / BLOB columns the writer FSST-compresses: l_comment text, short
    and empty strings, strings longer than 255 bytes, random binary bytes
    (every byte value, zeros included), NULLs (written as empty strings)."""
    words = [b"carefully", b"regular", b"deposits", b"haggle", b"ironic", b" ", b"the", b"quickly", b"final", b"."]
    text = [b" ".join(words[j] for j in rng.integers(0, len(words), rng.integers(1, 9))) for _ in range(n)]
    short = [bytes(rng.integers(97, 100, rng.integers(0, 4), dtype=np.uint8)) for _ in range(n)]
    long = [b"x" * int(rng.integers(0, 600)) + bytes(rng.integers(97, 123, 7, dtype=np.uint8)) for _ in range(n)]
    binary = [bytes(rng.integers(0, 256, rng.integers(0, 40), dtype=np.uint8)) for _ in range(n)]
    nulls = [None if i % 5 == 0 else text[i] for i in range(n)]
    return [("text", fl.VARCHAR, text, fl.ENC_FSST), ("short", fl.VARCHAR, short, fl.ENC_FSST),
            ("long", fl.VARCHAR, long, fl.ENC_FSST), ("bin", fl.BLOB, binary, fl.ENC_FSST),
            ("nulls", fl.VARCHAR, nulls, fl.ENC_FSST), ("auto", fl.VARCHAR, text, fl.ENC_AUTO)]


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{}, {"FLS_FSST_MAX_SYMBOLS": "8"}, {"FLS_FSST_MAX_LEN": "8"},
                                 {"FLS_FSST_MAX_SYMBOLS": "0"}])
@pytest.mark.parametrize("n,rowgroup", [(20000, 4096), (1, 65536), (3000, 1024)])
def test_gpu_writer_fsst_bytes_identical(fl, gpu, monkeypatch, env, n, rowgroup):
    """FSST chunks compressed on the GPU (fls_writer_set_device: the host builds
    the table, the GPU applies the greedy longest match) are byte-identical to
    the host compressor's, escapes (small tables) and 8-byte symbols included."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    cols = _fsst_columns(fl, n, np.random.default_rng(n))
    cpu = fl.write_image(cols, rowgroup=rowgroup).tobytes()
    dev = fl.write_image(cols, rowgroup=rowgroup, device=0, threads=4).tobytes()
    assert len(cpu) == len(dev)
    assert cpu == dev
    monkeypatch.setenv("FLS_WRITER_FSST_GPU", "0")   # the knob that keeps FSST on the host
    assert fl.write_image(cols, rowgroup=rowgroup, device=0).tobytes() == cpu


@pytest.mark.gpu
def test_gpu_writer_fsst_lineitem_comment_decodes(fl, ref, gpu):
    """l_comment through the GPU compressor: byte-identical to the host's and
    decoded exactly by the GPU scan."""
    from helpers import assert_column_equal, gpu_decode_all
    n = 65536 * 2 + 100
    ss = fl.gen_strings("lineitem_full", 15, 0, n, scale=1)
    cols = [("l_comment", fl.VARCHAR, ss, fl.ENC_FSST)]
    img = fl.write_image(cols, device=0, threads=8)
    assert img.tobytes() == fl.write_image(cols).tobytes()
    t, st, out = gpu_decode_all(fl, img)
    assert_column_equal(fl, ref.RefFile(img), 0, out[0], img.ptr)


def _add_rg(fl, w, ints, strs):
    """one row group of (INTEGER, VARCHAR) straight through the C-ABI writer"""
    import ctypes as C
    o = np.zeros(len(strs) + 1, dtype=np.uint32)
    o[1:] = np.cumsum([len(s) for s in strs])
    buf = np.frombuffer(b"".join(strs) or b"\0", dtype=np.uint8).copy()
    ints = np.ascontiguousarray(ints, dtype=np.int32)
    data = (C.c_void_p * 2)(ints.ctypes.data, buf.ctypes.data)
    offs = (C.c_void_p * 2)(None, o.ctypes.data)
    return fl.lib.fls_writer_add_rowgroup(w, len(ints), data, offs)


@pytest.mark.gpu
def test_gpu_writer_fsst_failure_marks_writer_failed(fl, gpu, monkeypatch):
    """a failed GPU FSST compression drops its segment's
    row groups while the GPU encoder's batch still holds the integer column's
    jobs for them.  The writer is then marked failed: a later add or finish
    returns an error instead of completing those jobs into row groups that do
    not exist (heap corruption) or into the wrong ones."""
    import ctypes as C
    rng = np.random.default_rng(5)
    n = 4096
    strs = [s.encode() for s in fsst_text(n, rng)]
    w = fl.lib.fls_writer_new(0)
    try:
        assert fl.lib.fls_writer_set_rowgroup_size(w, n) == 0
        assert fl.lib.fls_writer_set_device(w, 0) == 0
        assert fl.lib.fls_writer_add_column(w, b"i", fl.INT32, 0, 0, fl.ENC_FFOR) == 0
        assert fl.lib.fls_writer_add_column(w, b"s", fl.VARCHAR, 0, 0, fl.ENC_FSST) == 0
        ints = rng.integers(0, 1000, n)
        assert _add_rg(fl, w, ints, strs) == 0          # a healthy row group in the GPU batch
        monkeypatch.setenv("FLS_TEST_FAIL_FSST_GPU", "1")
        assert _add_rg(fl, w, ints, strs) < 0           # its FSST chunk fails on the device
        assert b"injected" in fl.lib.fls_last_error()
        monkeypatch.delenv("FLS_TEST_FAIL_FSST_GPU")
        assert _add_rg(fl, w, ints, strs) < 0           # the writer stays failed
        assert b"failed earlier" in fl.lib.fls_last_error()
        p, ln = C.c_void_p(), C.c_uint64()
        assert fl.lib.fls_writer_finish_image(w, C.byref(p), C.byref(ln)) < 0
        assert b"failed earlier" in fl.lib.fls_last_error()
    finally:
        fl.lib.fls_writer_free(w)


@pytest.mark.gpu
@pytest.mark.parametrize("pipelined", [0, 1])
def test_gpu_encoder_failure_marks_writer_failed(fl, gpu, monkeypatch, pipelined):
    """A GPU encoder set that comes back without one of its chunks (injected:
    FLS_TEST_FAIL_GPU_ENCODE) fails the call that completes it, names the row
    group and column, and leaves the writer failed: no later finish writes a
    file whose row groups miss chunks -- also with pipelined calls (the
    pending row group is appended before the set completes)."""
    import ctypes as C
    rng = np.random.default_rng(6)
    n = 4096
    strs = [b"x%d" % (i % 7) for i in range(n)]
    w = fl.lib.fls_writer_new(0)
    try:
        assert fl.lib.fls_writer_set_rowgroup_size(w, n) == 0
        assert fl.lib.fls_writer_set_device(w, 0) == 0
        assert fl.lib.fls_writer_add_column(w, b"i", fl.INT32, 0, 0, fl.ENC_FFOR) == 0
        assert fl.lib.fls_writer_add_column(w, b"s", fl.VARCHAR, 0, 0, fl.ENC_AUTO) == 0
        assert fl.lib.fls_writer_set_pipelined(w, pipelined) == 0
        # (the buffers live to the end: a pipelined call's tasks read them later)
        ints = np.ascontiguousarray(rng.integers(0, 1000, n), dtype=np.int32)
        o = np.zeros(n + 1, dtype=np.uint32)
        o[1:] = np.cumsum([len(x) for x in strs])
        buf = np.frombuffer(b"".join(strs), dtype=np.uint8).copy()
        data = (C.c_void_p * 2)(ints.ctypes.data, buf.ctypes.data)
        offs = (C.c_void_p * 2)(None, o.ctypes.data)
        assert fl.lib.fls_writer_add_rowgroup(w, n, data, offs) == 0
        monkeypatch.setenv("FLS_TEST_FAIL_GPU_ENCODE", "1")
        p, ln = C.c_void_p(), C.c_uint64()
        assert fl.lib.fls_writer_finish_image(w, C.byref(p), C.byref(ln)) < 0
        assert b"no chunk for row group" in fl.lib.fls_last_error()
        monkeypatch.delenv("FLS_TEST_FAIL_GPU_ENCODE")
        assert fl.lib.fls_writer_finish_image(w, C.byref(p), C.byref(ln)) < 0
        assert b"failed earlier" in fl.lib.fls_last_error()
    finally:
        fl.lib.fls_writer_free(w)


# ---- DICT chunks of integer columns on the GPU (dict_analyze_kernel /
# dict_encode_kernel; SURVEY.md 8(f) row 1 "dict analysis";
# reference writer stub src/writer/write_fastlane_stream.cpp:65-107,294-314) ----
def _dict_columns(fl, n, rng):
    """Explicit ENC_DICT and DICT-choosing ENC_AUTO columns of every integer
    type: a few distinct values over the whole range (the type's min and max,
    0, and the all-ones value -- for 64-bit types the GPU table's empty marker,
    kept beside the table), a single value, and, for wide types, more distinct
    values than dict_encode_kernel sorts in LDS (kDictGpuMax = 16,384: those
    chunks go back to the host, same bytes)."""
    cols = []
    for tn in INT_TYPES:
        ty = getattr(fl, tn)
        dt = np.dtype(fl.NP_DTYPE[ty])
        info = np.iinfo(dt)
        pool = rng.integers(info.min, info.max, 40, dtype=dt, endpoint=True)
        pool[:4] = [info.min, info.max, 0, np.array(-1).astype(dt) if info.min < 0 else info.max]
        few = pool[rng.integers(0, 40, n)]
        one = np.full(n, pool[7], dtype=dt)
        cols += [(f"{tn}_dict_few", ty, few, fl.ENC_DICT), (f"{tn}_dict_one", ty, one, fl.ENC_DICT),
                 (f"{tn}_auto_few", ty, few[::-1].copy(), fl.ENC_AUTO)]
        if dt.itemsize >= 4:
            wide = rng.integers(info.min, info.max, 20000, dtype=dt, endpoint=True)
            cols += [(f"{tn}_dict_many", ty, wide[rng.integers(0, 20000, n)], fl.ENC_DICT)]
    return cols


def test_dict_columns_are_dict_on_cpu(fl):
    cols = _dict_columns(fl, 20000, np.random.default_rng(3))
    encs = _chunk_encodings(fl.write_image(cols, rowgroup=4096).tobytes())
    assert set(encs) == {fl.ENC_DICT}, encs


@pytest.mark.gpu
@pytest.mark.parametrize("n,rowgroup", [(65536 * 2 + 777, 65536), (20000, 4096), (1024 * 3 + 5, 1024), (1, 65536)])
def test_gpu_writer_dict_bytes_identical(fl, ref, gpu, monkeypatch, n, rowgroup):
    """DICT chunks of every integer type encoded on the GPU -- the distinct
    values hashed and sorted by signed value, the codes FFOR-packed -- and
    ENC_AUTO's DICT estimate made on the GPU (the CPU writer's sample rule and
    size estimate): the file is the CPU writer's, byte for byte, decodes to
    the input under the oracle, and so is the round-3 path (host estimate and
    host DICT encoding, FLS_WRITER_DICT_GPU=0)."""
    cols = _dict_columns(fl, n, np.random.default_rng(n + 3))
    cpu_img = fl.write_image(cols, rowgroup=rowgroup)
    cpu = cpu_img.tobytes()
    dev = fl.write_image(cols, rowgroup=rowgroup, device=0, threads=8).tobytes()
    assert len(cpu) == len(dev)
    assert cpu == dev
    rf = ref.RefFile(cpu_img)
    for c, (name, ty, vals, _) in enumerate(cols):
        got = np.concatenate([rf.decode(c, r) for r in range(rf.nrowgroups)])
        assert np.array_equal(got.view(vals.dtype), vals), name
    monkeypatch.setenv("FLS_WRITER_DICT_GPU", "0")
    assert fl.write_image(cols, rowgroup=rowgroup, device=0).tobytes() == cpu


@pytest.mark.gpu
def test_gpu_writer_auto_dict_estimate_matches_host(fl, gpu, monkeypatch):
    """ENC_AUTO on the GPU without the host's sample: chunks near the DICT
    boundaries (sample of 1,024 with ~512 distinct values, distinct counts
    around the FFOR / DICT break-even) choose exactly what the CPU writer
    chooses."""
    rng = np.random.default_rng(77)
    n = 65536 * 3
    cols = []
    for k in (400, 500, 512, 520, 600, 3000, 9000, 30000):
        pool = rng.integers(-2**62, 2**62, k)
        cols.append((f"i64_{k}", fl.INT64, pool[rng.integers(0, k, n)], fl.ENC_AUTO))
        pool32 = rng.integers(-2**30, 2**30, k)
        cols.append((f"i32_{k}", fl.INT32, pool32[rng.integers(0, k, n)].astype(np.int32), fl.ENC_AUTO))
    cpu = fl.write_image(cols).tobytes()
    assert fl.ENC_DICT in _chunk_encodings(cpu) and fl.ENC_FFOR in _chunk_encodings(cpu)
    assert fl.write_image(cols, device=0, threads=8).tobytes() == cpu


def _str_dict_columns(fl, n, rng):
    """VARCHAR / BLOB columns for the GPU string dictionary: few distinct
    strings (l_shipmode-like), empty strings and NULLs, binary bytes (NUL,
    0xFF), distinct counts around ENC_AUTO's n / 8 limit, more distinct
    strings than the GPU sorts (kDictGpuMax: the host builds that one) and
    free text (AUTO: past the limit, FSST)."""
    modes = [b"AIR", b"FOB", b"MAIL", b"RAIL", b"REG AIR", b"SHIP", b"TRUCK"]
    few = [modes[k] for k in rng.integers(0, 7, n)]
    bins = [bytes(rng.integers(0, 256, rng.integers(0, 6), dtype=np.uint8)) for _ in range(23)]
    binary = [bins[k] for k in rng.integers(0, 23, n)]
    nulls = [None if i % 7 == 0 else few[i] for i in range(n)]
    near = max(1, n // 8)
    around = [b"k%d" % k for k in rng.integers(0, near, n)]          # distinct count just under n / 8
    over = [b"k%d" % k for k in rng.integers(0, near + near // 2 + 2, n)]
    many = [b"m%06d" % k for k in rng.integers(0, 20000, n)]
    text = [b"t%d %s" % (i, b"x" * int(i % 13)) for i in range(n)]
    return [("few_dict", fl.VARCHAR, few, fl.ENC_DICT), ("few_auto", fl.VARCHAR, few[::-1], fl.ENC_AUTO),
            ("bin_dict", fl.BLOB, binary, fl.ENC_DICT), ("bin_auto", fl.BLOB, binary, fl.ENC_AUTO),
            ("nulls_auto", fl.VARCHAR, nulls, fl.ENC_AUTO), ("around_auto", fl.VARCHAR, around, fl.ENC_AUTO),
            ("over_auto", fl.VARCHAR, over, fl.ENC_AUTO), ("many_dict", fl.VARCHAR, many, fl.ENC_DICT),
            ("text_auto", fl.VARCHAR, text, fl.ENC_AUTO)]


@pytest.mark.gpu
@pytest.mark.parametrize("n,rowgroup", [(65536 * 2 + 777, 65536), (20000, 4096), (9, 1024), (1, 65536)])
def test_gpu_writer_str_dict_bytes_identical(fl, ref, gpu, monkeypatch, n, rowgroup):
    """VARCHAR / BLOB dictionaries built on the GPU (str_dict_kernel: the
    distinct strings in order of first appearance, every row's code, ENC_AUTO's
    limit of n / 8 distinct strings): the file is the CPU writer's, byte for
    byte, and its strings decode under the oracle; the host build
    (FLS_WRITER_DICT_GPU=0) writes the same file.  FLS_WRITER_STRDICT_GPU=1
    selects the GPU build (off by default: one round trip per chunk measured
    slower than the host threads' build in COPY)."""
    cols = _str_dict_columns(fl, n, np.random.default_rng(n + 11))
    cpu_img = fl.write_image(cols, rowgroup=rowgroup)
    cpu = cpu_img.tobytes()
    monkeypatch.setenv("FLS_WRITER_STRDICT_GPU", "1")   # opt-in (the host build is the default)
    dev = fl.write_image(cols, rowgroup=rowgroup, device=0, threads=8).tobytes()
    assert len(cpu) == len(dev)
    assert cpu == dev
    rf = ref.RefFile(cpu_img)
    for c, (name, _, vals, _) in enumerate(cols):
        assert rf.strings_column(c) == [b"" if v is None else v for v in vals], name
    monkeypatch.setenv("FLS_WRITER_DICT_GPU", "0")
    assert fl.write_image(cols, rowgroup=rowgroup, device=0).tobytes() == cpu


def test_str_dict_columns_cover_dict_and_fsst_cpu(fl):
    cols = _str_dict_columns(fl, 65536, np.random.default_rng(4))
    encs = _chunk_encodings(fl.write_image(cols).tobytes())
    assert encs.get(fl.ENC_DICT, 0) >= 6 and encs.get(fl.ENC_FSST, 0) >= 2, encs


def _alp_columns(fl, n, rng):
    """FLOAT / DOUBLE columns that exercise ALP's choices: decimals (one
    exponent fits), integers as doubles, values with no decimal form (every
    value an exception), specials (NaN, +-inf, -0.0, subnormals, huge), a
    constant, float32 twins, and NULLs (placeholders: the previous value)."""
    price = np.round(rng.random(n) * 1e5, 2)
    ints = rng.integers(-10**6, 10**6, n).astype(np.float64)
    rnd = rng.standard_normal(n)
    special = np.round(rng.random(n) * 100, 1)
    k = np.arange(n)
    for j, x in enumerate([np.nan, np.inf, -np.inf, -0.0, 5e-324, 1e300, 0.0]):
        special[k % 97 == j] = x
    const = np.full(n, 3.14)
    mixed = np.where(rng.random(n) < 0.3, rnd, price)   # some vectors mostly exceptions
    fprice = np.round(rng.random(n) * 1e3, 2).astype(np.float32)
    frnd = rng.standard_normal(n).astype(np.float32)
    with np.errstate(over="ignore"):
        fspecial = special.astype(np.float32)                # 1e300 -> inf
    fspecial[k % 89 == 3] = np.float32(1e-40)               # float32 subnormals (no flush to zero)
    fspecial[k % 89 == 4] = np.float32(-3e-42)
    masked = np.ma.masked_array(np.round(rng.random(n) * 50, 3), mask=rng.random(n) < 0.2)
    return [("price", fl.DOUBLE, price, fl.ENC_ALP), ("ints", fl.DOUBLE, ints, fl.ENC_AUTO),
            ("rnd", fl.DOUBLE, rnd, fl.ENC_ALP), ("special", fl.DOUBLE, special, fl.ENC_ALP),
            ("const", fl.DOUBLE, const, fl.ENC_AUTO), ("mixed", fl.DOUBLE, mixed, fl.ENC_ALP),
            ("fprice", fl.FLOAT, fprice, fl.ENC_ALP), ("frnd", fl.FLOAT, frnd, fl.ENC_AUTO),
            ("fspecial", fl.FLOAT, fspecial, fl.ENC_ALP), ("masked", fl.DOUBLE, masked, fl.ENC_ALP)]


@pytest.mark.gpu
@pytest.mark.parametrize("n,rowgroup", [(65536 * 2 + 777, 65536), (20000, 4096), (1024 * 3 + 5, 1024), (9, 1024),
                                        (1, 65536)])
def test_gpu_writer_alp_bytes_identical(fl, ref, gpu, monkeypatch, n, rowgroup):
    """ALP chunks of FLOAT / DOUBLE columns encoded on the GPU
    (alp_encode_kernel: the sampled (e, f) votes, each vector's cheapest
    candidate, exceptions and FFOR packing): the file -- chunks and float zone
    maps -- is the CPU writer's, byte for byte, its values decode bit-exactly
    under the oracle, and the host path (the default since round 5;
    FLS_WRITER_ALP_GPU=1 opts into the GPU) writes the same."""
    cols = _alp_columns(fl, n, np.random.default_rng(n + 5))
    cpu_img = fl.write_image(cols, rowgroup=rowgroup)
    cpu = cpu_img.tobytes()
    monkeypatch.setenv("FLS_WRITER_ALP_GPU", "1")
    dev = fl.write_image(cols, rowgroup=rowgroup, device=0, threads=8).tobytes()
    assert len(cpu) == len(dev)
    assert cpu == dev
    rf = ref.RefFile(cpu_img)
    for c, (name, ty, vals, _) in enumerate(cols):
        got = np.concatenate([rf.decode(c, r) for r in range(rf.nrowgroups)])
        want = np.ma.getdata(vals)
        if np.ma.isMaskedArray(vals):  # NULL rows hold the previous valid value
            m = np.ma.getmaskarray(vals)
            want = want.copy()
            for i in np.flatnonzero(m):
                want[i] = want[i - 1] if i > 0 else 0.0
            keep = ~m
            assert np.array_equal(got.view(want.dtype)[keep].view(np.uint8), want[keep].view(np.uint8)), name
        else:
            assert np.array_equal(got, want.view(np.uint8)), name
    monkeypatch.delenv("FLS_WRITER_ALP_GPU")
    assert fl.write_image(cols, rowgroup=rowgroup, device=0).tobytes() == cpu


@pytest.mark.gpu
def test_gpu_writer_alp_lineitem_dbl_decodes(fl, gpu, monkeypatch):
    """lineitem with the four DECIMAL columns as DOUBLE (the lineitem_dbl
    workload's shape), written on the GPU (FLS_WRITER_ALP_GPU=1): the file is
    the CPU writer's and the GPU decode of it returns every value's bits."""
    monkeypatch.setenv("FLS_WRITER_ALP_GPU", "1")
    n = 65536 + 1000
    rng = np.random.default_rng(11)
    qty = rng.integers(1, 51, n).astype(np.float64)
    price = np.round(rng.integers(90000, 10500000, n) / 100.0, 2)
    disc = rng.integers(0, 11, n) / 100.0
    tax = rng.integers(0, 9, n) / 100.0
    cols = [("q", fl.DOUBLE, qty, fl.ENC_ALP), ("p", fl.DOUBLE, price, fl.ENC_ALP),
            ("d", fl.DOUBLE, disc, fl.ENC_ALP), ("t", fl.DOUBLE, tax, fl.ENC_AUTO)]
    cpu = fl.write_image(cols).tobytes()
    img = fl.write_image(cols, device=0, threads=4)
    assert img.tobytes() == cpu
    t = fl.Connection([0]).read_image(img)
    got = {c: [] for c in range(len(cols))}
    for _, arrs in t.scan(cols=list(range(len(cols)))):
        for c in got:
            got[c].append(np.asarray(arrs[c]).view(np.uint8))
    for c, (_, _, vals, _) in enumerate(cols):
        assert np.array_equal(np.concatenate(got[c]), vals.view(np.uint8)), c
