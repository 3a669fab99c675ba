"""ALP (FLOAT/DOUBLE) and FSST (VARCHAR) -- SURVEY.md 8(f) row 3, the FP and
string decoders inside RowgroupReader::materialize() (reference
src/fastlanes_facade.cpp:48, consumers flt_col_t / dbl_col_t / FLSStrColumn at
:140-170).

CPU tests: the writer's encodings round-trip bit-exactly through the oracle
(oracle/flsref.c decodes ALP and FSST independently of the encoder), the
format invariants hold (exceptions, escapes, heap layout), and corrupt chunks
are rejected on open.  GPU tests: the HIP ALP path (decode kernel) and the FSST
kernel produce the oracle's bytes / strings exactly, device-resident and
through the scan pipeline."""
import struct

import numpy as np
import pytest

from helpers import fsst_text, special_doubles


def bits(a):
    return np.ascontiguousarray(a).view(np.uint8)


@pytest.mark.parametrize("kind", ["price", "ratio", "mixed", "ints", "tiny", "float1", "float_rand"])
def test_alp_roundtrip_bit_exact(fl, ref, kind):
    rng = np.random.default_rng(hash(kind) % 2**32)
    n = 70001
    if kind == "price":
        v = np.round(rng.uniform(900, 105000, n), 2)
    elif kind == "ratio":
        v = rng.random(n)                                  # mostly exceptions (no decimal form)
    elif kind == "mixed":
        v = np.round(rng.normal(0, 1e4, n), 3)
        v[rng.integers(0, n, 500)] = special_doubles(500, rng)
    elif kind == "ints":
        v = rng.integers(-2**40, 2**40, n).astype(np.float64)
    elif kind == "tiny":
        v = np.round(rng.uniform(0, 1, n), 5) * 1e-6
    elif kind == "float1":
        v = np.round(rng.uniform(-100, 100, n), 1).astype(np.float32)
    else:
        v = rng.standard_normal(n).astype(np.float32)
    ty = fl.FLOAT if v.dtype == np.float32 else fl.DOUBLE
    img = fl.write_image([("v", ty, v, fl.ENC_ALP)])
    rf = ref.RefFile(img)
    got = rf.decode_column(0)
    assert np.array_equal(got, bits(v))


def test_alp_compresses_decimals(fl):
    rng = np.random.default_rng(5)
    v = np.round(rng.uniform(900, 105000, 65536), 2)      # l_extendedprice-like
    img = fl.write_image([("p", fl.DOUBLE, v, fl.ENC_AUTO)])
    assert len(img.tobytes()) < 0.45 * v.nbytes         # ~24 bits/value vs 64


def _chunk_header(raw, col=0, rg=0):
    """(offset, header fields) of a chunk via the footer."""
    foot, flen = struct.unpack_from("<QI", raw, len(raw) - 16)
    ncols = struct.unpack_from("<I", raw, foot + 4)[0]
    p = foot + 32
    for _ in range(ncols):
        p += 6 + struct.unpack_from("<H", raw, p + 4)[0]
    p += rg * (4 + 16 * ncols)
    off = struct.unpack_from("<Q", raw, p + 4 + 16 * col)[0]
    return off


def test_alp_exception_layout(fl, ref):
    v = np.full(1024, 12.25)
    v[[3, 700]] = [np.nan, -0.0]
    raw = fl.write_image([("v", fl.DOUBLE, v, fl.ENC_ALP)]).tobytes()
    off = _chunk_header(raw)
    enc, T = raw[off + 4], raw[off + 5]
    meta = struct.unpack_from("<QqQHBBI", raw, off + 64)
    aux_count = meta[6]
    assert (enc, T) == (5, 64)
    assert aux_count & 0xFFFF == 2 and meta[4] == 0      # two exceptions, constant ints -> W=0
    e, f = (aux_count >> 16) & 0xFF, aux_count >> 24
    assert f <= e and 12.25 * 10 ** (e - f) == round(12.25 * 10 ** (e - f))


@pytest.mark.parametrize("n", [1, 1023, 1025, 65536, 70000])
def test_fsst_roundtrip_and_escapes(fl, ref, n):
    rng = np.random.default_rng(n)
    s = fsst_text(n, rng)
    # strings the symbol table cannot cover: raw bytes -> escapes (incl. 0xFF)
    for i in range(0, n, 97):
        s[i] = bytes(rng.integers(0, 256, rng.integers(0, 30), dtype=np.uint8).tolist())
    if n > 3:
        s[1] = b""
        s[2] = b"\xff" * 20
    img = fl.write_image([("c", fl.VARCHAR, s, fl.ENC_FSST)])
    rf = ref.RefFile(img)
    assert rf.strings_column(0) == [x if isinstance(x, bytes) else x.encode() for x in s]


def test_fsst_compresses_text(fl):
    rng = np.random.default_rng(9)
    s = fsst_text(65536, rng)
    img = fl.write_image([("c", fl.VARCHAR, s, fl.ENC_AUTO)])   # AUTO -> FSST (high cardinality)
    raw = img.tobytes()
    assert raw[_chunk_header(raw) + 4] == 7
    assert len(raw) < 0.5 * sum(map(len, s))


def test_varchar_auto_picks_dict_for_low_cardinality(fl):
    s = ["AIR", "MAIL", "SHIP"] * 10000
    raw = fl.write_image([("c", fl.VARCHAR, s, fl.ENC_AUTO)]).tobytes()
    assert raw[_chunk_header(raw) + 4] == 3


@pytest.mark.parametrize("wl", ["lineitem_full", "lineitem_dbl"])
def test_full_fidelity_workloads_match_generator(fl, ref, wl):
    """lineitem with l_comment (FSST, TPC-H grammar text) and with the DECIMAL
    columns as DOUBLE (ALP): the oracle decodes the generator's values."""
    img = fl.gen_image(wl, 0.01)
    rf = ref.RefFile(img)
    n = rf.nrows
    assert n == 60175
    for c in range(rf.ncols):
        name, ty, _, _ = rf.column(c)
        if ty == fl.VARCHAR:
            assert rf.strings_column(c) == fl.gen_strings(wl, c, 0, n, 0.01), name
        else:
            dt = fl.NP_DTYPE[ty]
            assert np.array_equal(rf.decode_column(c).view(dt), fl.gen_values(wl, c, 0, n, dt, 0.01)), name
    if wl == "lineitem_full":
        lens = [len(x) for x in fl.gen_strings(wl, 15, 0, 5000, 0.01)]
        assert min(lens) == 10 and max(lens) == 43


def test_corrupt_alp_and_fsst_rejected(fl, ref):
    v = np.round(np.arange(5000) * 0.25, 2)
    raw = bytearray(fl.write_image([("v", fl.DOUBLE, v, fl.ENC_ALP)]).tobytes())
    off = _chunk_header(raw)
    struct.pack_into("<I", raw, off + 64 + 28, (30 << 16) | 1)   # exponent 30 > 18
    with pytest.raises(fl.FlsError, match="ALP exponent"):
        fl.Connection().read_image(bytes(raw))
    s = fsst_text(3000, np.random.default_rng(1))
    raw = bytearray(fl.write_image([("c", fl.VARCHAR, s, fl.ENC_FSST)]).tobytes())
    off = _chunk_header(raw)
    aux = struct.unpack_from("<Q", raw, off + 32)[0]
    raw[off + aux + 2048] = 9                                   # symbol length 9
    with pytest.raises(fl.FlsError, match="FSST symbol length"):
        fl.Connection().read_image(bytes(raw))


# ---- GPU ---------------------------------------------------------------------
from helpers import assert_column_equal, assert_strings_equal, gpu_decode_all  # noqa: E402


def _mixed_table(fl, n, seed):
    rng = np.random.default_rng(seed)
    price = np.round(rng.uniform(900, 105000, n), 2)
    mixed = np.round(rng.normal(0, 1e4, n), 3)
    mixed[rng.integers(0, n, max(1, n // 100))] = special_doubles(max(1, n // 100), rng)
    ratio = rng.random(n)
    f32 = np.round(rng.uniform(-100, 100, n), 1).astype(np.float32)
    fr = rng.standard_normal(n).astype(np.float32)
    text = fsst_text(n, rng)
    for i in range(0, n, 211):
        text[i] = bytes(rng.integers(0, 256, rng.integers(0, 40), dtype=np.uint8).tolist())
    cols = [("price", fl.DOUBLE, price, fl.ENC_ALP), ("mixed", fl.DOUBLE, mixed, fl.ENC_ALP),
            ("ratio", fl.DOUBLE, ratio, fl.ENC_ALP), ("f32", fl.FLOAT, f32, fl.ENC_ALP),
            ("frand", fl.FLOAT, fr, fl.ENC_ALP), ("comment", fl.VARCHAR, text, fl.ENC_FSST),
            ("key", fl.INT64, np.arange(n) * 3, fl.ENC_DELTA)]
    return fl.write_image(cols), cols


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 1000, 1024, 65536, 3 * 65536 + 4321])
def test_gpu_alp_fsst_device_resident(fl, ref, gpu, n):
    img, cols = _mixed_table(fl, n, n)
    t, st, out = gpu_decode_all(fl, img)
    rf = ref.RefFile(img)
    for c, (name, ty, vals, _) in enumerate(cols):
        assert_column_equal(fl, rf, c, out[c], img.ptr)
        if ty in (fl.FLOAT, fl.DOUBLE):
            assert np.array_equal(out[c], bits(vals)), name


# FSST kernels: the segmented one (default for files with segment tables,
# ring cap 4096 or 3072 bytes) and the round-2 code-parallel one (files
# without them, or FLS_FSST_SEG=0)
FSST_KERNELS = {"seg": {}, "seg3072": {"FLS_FSST_SEG_CAP": "3072"}, "cp": {"FLS_FSST_SEG": "0"},
                # the fused launch (fused_kernel: its FSST part)
                "fused": {"FLS_FUSED": "1"}}


def _use_kernel(monkeypatch, kernel):
    for k, v in FSST_KERNELS[kernel].items():
        monkeypatch.setenv(k, v)


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", list(FSST_KERNELS))
def test_gpu_fsst_escape_heavy_and_long_strings(fl, ref, gpu, monkeypatch, kernel):
    _use_kernel(monkeypatch, kernel)
    rng = np.random.default_rng(3)
    n = 20000
    s = []
    for i in range(n):
        k = i % 5
        if k == 0:
            s.append(b"")
        elif k == 1:
            s.append(b"\xff" * int(rng.integers(1, 50)))                           # escapes only
        elif k == 2:
            s.append(bytes(rng.integers(0, 256, int(rng.integers(1, 300)), dtype=np.uint8).tolist()))
        elif k == 3:
            s.append(("lorem ipsum dolor sit amet " * int(rng.integers(1, 200))).encode())  # up to 5 KB
        else:
            s.append(b"x" * 12)
    img = fl.write_image([("s", fl.VARCHAR, s, fl.ENC_FSST)])
    t, st, out = gpu_decode_all(fl, img)
    rf = ref.RefFile(img)
    assert_strings_equal(fl, rf, 0, out[0])


@pytest.mark.gpu
def test_gpu_alp_fsst_scan_pipeline(fl, ref, gpu, monkeypatch):
    monkeypatch.setenv("FLS_SCAN_BATCH", "3")
    n = 7 * 65536 + 999
    img, cols = _mixed_table(fl, n, 77)
    rf = ref.RefFile(img)
    conn = fl.Connection([0, 0])
    t = conn.read_image(img)
    seen = 0
    for first, got in t.scan(cols=[0, 4, 5]):
        rg = first // 65536
        assert np.array_equal(got[0], rf.decode(0, rg))
        assert np.array_equal(got[4], rf.decode(4, rg))
        assert fl.string_t_decode(got[5]) == rf.strings_rg(5, rg)
        seen += 1
    assert seen == rf.nrowgroups


@pytest.mark.gpu
@pytest.mark.parametrize("wl,split", [("lineitem_full", "default"), ("lineitem_full", None),
                                      ("lineitem_full", "0"), ("lineitem_full", "1,28"),
                                      ("lineitem_full", "4,1"), ("lineitem_full", "cu8"),
                                      ("lineitem_full", "cu24"), ("lineitem_dbl", None)],
                         ids=["full-default", "full-overlap", "full-serial", "full-fsst-wide", "full-fsst-narrow",
                              "full-cu-split8", "full-cu-split24", "dbl"])
def test_gpu_full_fidelity_lineitem(fl, ref, gpu, monkeypatch, wl, split):
    """Full-fidelity lineitem; with FSST columns the table decode overlaps the
    FSST kernels with the main one (launch_all): the default split, serial
    (FLS_OVERLAP_FSST_WPC=0) and extreme splits must all decode exactly.  At
    SF0.1 the default runs serially (fewer FSST vectors per CU than
    FLS_OVERLAP_MIN_VECS_PER_CU); the overlapped cases lower that threshold."""
    if split != "default":
        monkeypatch.setenv("FLS_OVERLAP_MIN_VECS_PER_CU", "0")
        monkeypatch.setenv("FLS_FUSED", "0")   # the overlapped kernels, not the fused one
    if split == "0":
        monkeypatch.setenv("FLS_OVERLAP_FSST_WPC", "0")
    elif split and split.startswith("cu"):   # CU-partitioned overlap (FLS_OVERLAP_CU_SPLIT)
        monkeypatch.setenv("FLS_OVERLAP_CU_SPLIT", split[2:])
    elif split and split != "default":
        bpc, wpc = split.split(",")
        monkeypatch.setenv("FLS_OVERLAP_DECODE_BPC", bpc)
        monkeypatch.setenv("FLS_OVERLAP_FSST_WPC", wpc)
    img = fl.gen_image(wl, 0.1)
    t, st, out = gpu_decode_all(fl, img)
    rf = ref.RefFile(img)
    for c in range(t.ncols):
        assert_column_equal(fl, rf, c, out[c], img.ptr)
    if wl == "lineitem_full":
        assert fl.string_t_decode(out[15][:16 * 3000]) == fl.gen_strings(wl, 15, 0, 3000, 0.1)


@pytest.mark.gpu
def test_gpu_fsst_corrupt_lengths_reported(fl, ref, gpu):
    s = fsst_text(5000, np.random.default_rng(4))
    raw = bytearray(fl.write_image([("c", fl.VARCHAR, s, fl.ENC_FSST)]).tobytes())
    off = _chunk_header(raw)
    struct.pack_into("<I", raw, off + 64 + 28, struct.unpack_from("<I", raw, off + 64 + 28)[0] + 5)
    t = fl.Connection().read_image(bytes(raw))
    t.device_upload()
    t.device_decode()
    with pytest.raises(fl.FlsError, match="corrupt"):
        t.device_sync()


def _boundary_strings():
    """With the table limited to {'a'*8}: string 0 is 1023 codes, string 1 the
    escape pair (255, 'Z') at compressed bytes 1023/1024 -- the escape is the
    last byte of decode round 0 and its literal the first of round 1, which has
    no other escape; then ordinary strings and more escapes across vectors."""
    s = [b"a" * (8 * 1023), b"Z"] + [b"a" * 8] * 300 + [b"aZa" * 5, b""] * 50
    s += [b"a" * (8 * 1022) + b"Z", b"QQ", b"a" * 16]      # escape pair straddling a string boundary
    return s


def test_fsst_escape_at_round_boundary_roundtrip(fl, ref, monkeypatch):
    monkeypatch.setenv("FLS_FSST_MAX_SYMBOLS", "1")
    s = _boundary_strings()
    img = fl.write_image([("s", fl.VARCHAR, s, fl.ENC_FSST)])
    assert ref.RefFile(img).strings_column(0) == s


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", list(FSST_KERNELS))
@pytest.mark.parametrize("maxsym", ["1", "8", "255"])
def test_gpu_fsst_escape_at_round_boundary(fl, ref, gpu, monkeypatch, maxsym, kernel):
    _use_kernel(monkeypatch, kernel)
    monkeypatch.setenv("FLS_FSST_MAX_SYMBOLS", maxsym)
    s = _boundary_strings() * 3
    img = fl.write_image([("s", fl.VARCHAR, s, fl.ENC_FSST)])
    t, st, out = gpu_decode_all(fl, img)
    assert fl.string_t_decode(out[0]) == s


# ---- FSST string-parallel kernel (chunks whose strings are <= 255 bytes) ----
def _sp_tables(fl, rng):
    """(name, strings) cases around the string-parallel kernel's eligibility:
    every string <= 255 bytes decompressed AND compressed, per chunk."""
    n = 70000
    text = fsst_text(n, rng)
    esc = [b"\xff" * int(k) for k in rng.integers(0, 128, 3000)]              # 2 compressed bytes per byte
    bin127 = [bytes(rng.integers(0, 256, int(k), dtype=np.uint8).tolist()) for k in rng.integers(0, 128, 3000)]
    edge = [b"", b"q", b"a" * 255, b"", b"lorem ipsum " * 21] * 300          # 255-byte strings, empties
    # row group 0 gets one 300-byte string (code-parallel), row group 1 stays short (string-parallel)
    mixed = fsst_text(65536, rng)
    mixed[777] = "long " * 60
    mixed += fsst_text(9000, rng)
    # ~8 decoded bytes per code: a round's output overruns the code-parallel
    # kernel's 2 KiB ring and is written in parts
    # (lengths in [192, 255] so the chunk's FFOR length bound stays <= 255)
    rep = [(b"abcdefgh" * 32)[: int(k)] for k in rng.integers(192, 249, 5000)]
    return [("text", text), ("escapes", esc), ("binary127", bin127), ("edge255", edge), ("repeat8", rep),
            ("mixed_rg", mixed)]


@pytest.mark.gpu
@pytest.mark.parametrize("policy", ["128", "0", "seg", "seg3072"],
                         ids=["string_parallel", "code_parallel", "segmented", "segmented3072"])
def test_gpu_fsst_string_and_code_parallel_agree(fl, ref, gpu, monkeypatch, capfd, policy):
    if policy.startswith("seg"):
        _use_kernel(monkeypatch, policy)
    else:
        monkeypatch.setenv("FLS_DECODE_POLICY", policy)
        _use_kernel(monkeypatch, "cp")
    monkeypatch.setenv("FLS_DEBUG", "1")
    for name, s in _sp_tables(fl, np.random.default_rng(21)):
        img = fl.write_image([("s", fl.VARCHAR, s, fl.ENC_FSST)])
        t, st, out = gpu_decode_all(fl, img)
        rf = ref.RefFile(img)
        assert_strings_equal(fl, rf, 0, out[0])
        err = capfd.readouterr().err
        # which kernels ran: chunks with segment tables (every file written
        # now) take the segmented kernel; without it (FLS_FSST_SEG=0) they are
        # code-parallel (u8 string lengths when all strings are <= 255 bytes),
        # and policy 128 sends those to the string-parallel kernel
        seg = policy.startswith("seg")
        assert ("fsst_sp_kernel" in err) == (policy == "128"), name
        assert ("fsst_kernel<8,small>" in err) == (policy == "0"), name
        assert ("fsst_kernel<8,any>" in err) == (name == "mixed_rg" and not seg), name
        assert ("fsst_kernel<16,small,seg>" in err) == seg, name
        assert ("fsst_kernel<16,any,seg>" in err) == (name == "mixed_rg" and seg), name


@pytest.mark.gpu
def test_gpu_fsst_string_parallel_scan_pipeline(fl, ref, gpu, monkeypatch):
    """Scan batches (balanced main kernel + string-parallel FSST) deliver the
    oracle's strings row group by row group."""
    monkeypatch.setenv("FLS_SCAN_BATCH", "2")
    img = fl.gen_image("lineitem_full", 0.05)
    rf = ref.RefFile(img)
    t = fl.Connection([0]).read_image(img)
    for first, got in t.scan(cols=[15]):
        assert fl.string_t_decode(got[15]) == rf.strings_rg(15, first // 65536)


def _fsst_vec0(raw):
    """(chunk offset, FsstVecHeader offset, comp_len, clen_w) of vector 0 of the first chunk."""
    off = _chunk_header(raw)
    aux_off = struct.unpack_from("<Q", raw, off + 32)[0]
    meta = off + struct.unpack_from("<Q", raw, off + 16)[0]
    vh = off + aux_off + struct.unpack_from("<Q", raw, meta + 16)[0]
    comp_len, _, clen_w = struct.unpack_from("<III", raw, vh + 4)
    return off, vh, comp_len, clen_w


def _seg_area(raw):
    _, vh, comp_len, clen_w = _fsst_vec0(raw)
    return vh + 16 + 128 * clen_w + ((comp_len + 15) & ~15), comp_len


@pytest.mark.gpu
@pytest.mark.parametrize("field", ["clen_base", "comp_len"])
@pytest.mark.parametrize("policy", ["128", "0", "seg"], ids=["string_parallel", "code_parallel", "segmented"])
def test_gpu_fsst_corrupt_compressed_lengths_reported(fl, ref, gpu, monkeypatch, field, policy):
    """A compressed-length stream that disagrees with the code stream (the
    string-parallel kernel's string starts) is clamped and reported by the
    string-parallel kernel.  The code-parallel and segmented kernels never
    read the per-string compressed lengths: they decode such a vector exactly,
    and report a code stream shortened under the strings' lengths (or the
    reader rejects it first, when the shorter stream no longer matches the
    segment table's count)."""
    if policy == "seg":
        _use_kernel(monkeypatch, "seg")
    else:
        monkeypatch.setenv("FLS_DECODE_POLICY", policy)
        _use_kernel(monkeypatch, "cp")
    s = fsst_text(5000, np.random.default_rng(6))
    img = fl.write_image([("c", fl.VARCHAR, s, fl.ENC_FSST)])
    raw = bytearray(img.tobytes())
    _, vh, comp_len, _ = _fsst_vec0(raw)
    if field == "comp_len" and comp_len % 16 == 1:
        pytest.skip("the shorter stream needs one segment fewer: rejected by the reader")
    at = vh + (8 if field == "clen_base" else 4)
    struct.pack_into("<I", raw, at, struct.unpack_from("<I", raw, at)[0] - 1)
    t = fl.Connection().read_image(bytes(raw))
    t.device_upload()
    t.device_decode()
    if field == "clen_base" and policy != "128":
        t.device_sync()
        assert_strings_equal(fl, ref.RefFile(img), 0, t.device_copy_out(0))
        return
    with pytest.raises(fl.FlsError, match="corrupt"):
        t.device_sync()


def test_fsst_segment_tables_written_and_pinned(fl, ref, monkeypatch):
    """Every FSST chunk carries a segment table (chunk header reserved0 = 16);
    the oracle recomputes it from the code stream with its own sequential
    state machine when it decodes, and rejects a table that disagrees."""
    monkeypatch.setenv("FLS_FSST_MAX_SYMBOLS", "8")           # escapes in the stream
    s = fsst_text(3000, np.random.default_rng(8)) + [b"\xff" * 7, b"Zz\x01" * 30] * 100
    s = [x if isinstance(x, bytes) else x.encode() for x in s]
    raw = bytearray(fl.write_image([("c", fl.VARCHAR, s, fl.ENC_FSST)]).tobytes())
    off = _chunk_header(raw)
    assert struct.unpack_from("<I", raw, off + 52)[0] == 16
    area, comp_len = _seg_area(raw)
    flags, nseg = struct.unpack_from("<II", raw, area)
    assert nseg == (comp_len + 15) // 16 and flags & 1 == 1
    segs = np.frombuffer(bytes(raw[area + 16: area + 16 + nseg]), np.uint8)
    assert (segs > 128).any()                                  # some segment starts with a literal
    assert ref.RefFile(bytes(raw)).strings_column(0) == s
    for k, delta in ((0, 1), (nseg // 2, -1)):
        bad = bytearray(raw)
        bad[area + 16 + k] = (bad[area + 16 + k] + delta) & 0xFF
        with pytest.raises(Exception):
            ref.RefFile(bytes(bad)).strings_column(0)
    bad = bytearray(raw)
    struct.pack_into("<I", bad, area, 0)                       # claims no escape codes
    with pytest.raises(Exception):
        ref.RefFile(bytes(bad)).strings_column(0)


@pytest.mark.gpu
@pytest.mark.parametrize("what", ["dlen_up", "dlen_down", "entry", "no_escape_flag"])
def test_gpu_fsst_corrupt_segment_table_reported(fl, ref, gpu, monkeypatch, what):
    """The segmented kernel checks every lane's decoded byte count against its
    segment's entry and every exit state against the next entry: a table that
    disagrees with the stream is reported, never silently decoded."""
    monkeypatch.setenv("FLS_FSST_MAX_SYMBOLS", "8")
    s = fsst_text(5000, np.random.default_rng(12)) + [b"\xffQ" * 9] * 200
    raw = bytearray(fl.write_image([("c", fl.VARCHAR, s, fl.ENC_FSST)]).tobytes())
    area, comp_len = _seg_area(raw)
    nseg = (comp_len + 15) // 16
    segs = raw[area + 16: area + 16 + nseg]
    if what == "dlen_up":
        k = next(i for i in range(nseg) if 0 < segs[i] < 128)
        raw[area + 16 + k] += 1
    elif what == "dlen_down":
        k = next(i for i in range(nseg) if 0 < segs[i] <= 128)
        raw[area + 16 + k] -= 1
    elif what == "entry":
        k = next(i for i in range(nseg) if segs[i] <= 120)
        raw[area + 16 + k] += 129                                 # claims a literal start
    else:
        struct.pack_into("<I", raw, area, 0)
    t = fl.Connection().read_image(bytes(raw))
    t.device_upload()
    t.device_decode()
    with pytest.raises(fl.FlsError, match="corrupt"):
        t.device_sync()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["381", "893", "1405", "2429", "0", "garbage"],
                         ids=["seg-nolean", "ablate-records", "ablate-flush", "ablate-write", "cp-v0", "not-a-number"])
def test_gpu_fsst_unknown_variant_refused(fl, gpu, monkeypatch, variant):
    """the product library holds the default FSST kernels
    only.  A tuning variable naming any other variant (the cost ablations,
    whose output is wrong by design, among them) fails the decode with
    FLS_ERR_CONFIG instead of silently running something else."""
    img = fl.write_image([("s", fl.VARCHAR, fsst_text(3000, np.random.default_rng(9)), fl.ENC_FSST)])
    t = fl.Connection().read_image(img)
    t.device_upload()
    monkeypatch.setenv("FLS_FSST_VARIANT", variant)
    with pytest.raises(fl.FlsError, match="FLS_FSST_VARIANT|not in this build") as ei:
        t.device_decode()
        t.device_sync()
    assert ei.value.code == -7
    monkeypatch.delenv("FLS_FSST_VARIANT")
    t.device_decode()
    t.device_sync()   # the default decodes again


@pytest.mark.gpu
@pytest.mark.parametrize("x", ["3", "5", "-1", "junk"])
def test_gpu_fused_x_refused_with_config_error(fl, gpu, monkeypatch, x):
    """a leftover FLS_FUSED_X (the fused kernel's experiment bits)
    fails a product-library decode with FLS_ERR_CONFIG, not a HIP error."""
    n = 70000
    rng = np.random.default_rng(4)
    img = fl.write_image([("k", fl.INT64, np.arange(n, dtype=np.int64), fl.ENC_DELTA),
                          ("s", fl.VARCHAR, fsst_text(n, rng), fl.ENC_FSST)])
    t = fl.Connection().read_image(img)
    t.device_upload()
    monkeypatch.setenv("FLS_FUSED_X", x)
    with pytest.raises(fl.FlsError, match="FLS_FUSED_X") as ei:
        t.device_decode()
        t.device_sync()
    assert ei.value.code == -7
    monkeypatch.delenv("FLS_FUSED_X")
    t.device_decode()
    t.device_sync()
    assert np.array_equal(t.device_copy_out(0).view(np.int64), np.arange(n, dtype=np.int64))


@pytest.mark.gpu
def test_gpu_stale_fsst_variant_does_not_fail_integer_tables(fl, gpu, monkeypatch):
    """the FSST variant check runs only for launches with FSST
    work, so a stale FLS_FSST_VARIANT cannot fail a table without strings
    (device-resident decode and the scan pipeline)."""
    x = np.arange(70000, dtype=np.int64) * 3
    img = fl.write_image([("x", fl.INT64, x, fl.ENC_DELTA)])
    monkeypatch.setenv("FLS_FSST_VARIANT", "893")
    t = fl.Connection().read_image(img)
    t.device_upload()
    t.device_decode()
    t.device_sync()
    assert np.array_equal(t.device_copy_out(0).view(np.int64), x)
    got = np.concatenate([cols[0].view(np.int64) for _, cols in t.scan()])
    assert np.array_equal(got, x)
