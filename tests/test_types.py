"""BOOLEAN, BLOB and CHAR: the reference's TypeMapping rows this path lacked
(/root/reference/src/type_mapping.cpp:13-14 BOOLEAN, :35-36 CHAR -> STR,
:40-42 BLOB -> BYTE_ARRAY; back again at :66-67, :89-90, :93-94).

Layout: BOOLEAN is a u8 column holding 0 / 1 (DuckDB's bool bytes), encoded
like UINT8 (FFOR packs it at W <= 1); BLOB is VARCHAR's layout and encodings
(DICT or FSST byte strings, decoded to 16-byte string_t); CHAR is written as
VARCHAR and reads back as VARCHAR, as in the reference.  CPU tests: the writer
and the oracle (oracle/flsref.c); GPU tests: the HIP decode through the C-ABI
vs the oracle, and COPY -> read_fastlanes / scan_fastlanes through the
extension."""
import numpy as np
import pytest

from ext_harness import Ext, ExtError
from helpers import assert_column_equal, gpu_decode_all


@pytest.fixture(scope="module")
def ext(_built):
    e = Ext()
    yield e
    e.close()


def _bools(n, rng):
    b = (rng.random(n) < 0.3).astype(np.uint8)
    b[: min(n, 2048)] = 1          # an all-true stretch: FFOR at W = 0
    return b


def _blobs(n, rng, distinct=None):
    """byte strings with NUL, 0xFF, quotes and backslashes, 0..40 bytes"""
    pool = None
    if distinct:
        pool = [bytes(rng.integers(0, 256, rng.integers(0, 30), dtype=np.uint8).tolist()) for _ in range(distinct)]
        pool[0] = b""
        pool[1] = b"\x00\xff'\"\\"
        return [pool[i] for i in rng.integers(0, distinct, n)]
    out = [bytes(rng.integers(0, 256, rng.integers(0, 41), dtype=np.uint8).tolist()) for _ in range(n)]
    out[0] = b""
    return out


def _table(fl, n, seed):
    rng = np.random.default_rng(seed)
    b = _bools(n, rng)
    cols = [("b_ffor", fl.BOOLEAN, b, fl.ENC_FFOR), ("b_auto", fl.BOOLEAN, b[::-1].copy(), fl.ENC_AUTO),
            ("x_fsst", fl.BLOB, _blobs(n, rng), fl.ENC_FSST), ("x_dict", fl.BLOB, _blobs(n, rng, 37), fl.ENC_DICT),
            ("x_auto", fl.BLOB, _blobs(n, rng, 5), fl.ENC_AUTO), ("k", fl.INT64, np.arange(n), fl.ENC_DELTA)]
    return fl.write_image(cols), cols


@pytest.mark.parametrize("n", [1, 1500, 2 * 65536 + 77])
def test_boolean_blob_written_and_oracle_decodes_cpu(fl, ref, n):
    img, cols = _table(fl, n, 7 + n)
    rf = ref.RefFile(img)
    assert [rf.column(c)[1] for c in range(len(cols))] == [9, 9, 21, 21, 21, 4]
    for c, (name, ty, vals, _) in enumerate(cols):
        if ty == fl.BLOB:
            assert rf.strings_column(c) == list(vals), name
        elif ty == fl.BOOLEAN:
            got = np.concatenate([rf.decode(c, g) for g in range(rf.nrowgroups)]).view(np.uint8)
            assert np.array_equal(got, vals), name


def test_boolean_bytes_must_be_zero_or_one_cpu(fl):
    with pytest.raises(fl.FlsError, match="BOOLEAN bytes must be 0 or 1"):
        fl.write_image([("b", fl.BOOLEAN, np.array([0, 1, 2], dtype=np.uint8), fl.ENC_FFOR)])
    with pytest.raises(fl.FlsError, match="FSST needs VARCHAR/BLOB"):
        fl.write_image([("b", fl.BOOLEAN, np.array([0, 1], dtype=np.uint8), fl.ENC_FSST)])


def _blob_hex(b):
    return b.hex()


def _duck_blob(b):
    """DuckDB's BLOB -> VARCHAR rendering (Blob::ToString)"""
    return "".join(chr(c) if 32 <= c <= 126 and chr(c) not in "\\'\"" else "\\x%02X" % c for c in b)


def _copy_types(ext, tmpfile, n, threads=1, name="types.fls"):
    rng = np.random.default_rng(n)
    b = [bool(x) for x in _bools(n, rng)]
    x = _blobs(n, rng, 11)
    ch = [f"c{i % 5}" * (i % 4) for i in range(n)]
    dst = tmpfile(name)
    cols = [("b", "BOOLEAN", ["true" if v else "false" for v in b]), ("x", "BLOB", [_blob_hex(v) for v in x]),
            ("c", "CHAR", ch), ("k", "BIGINT", list(range(n)))]
    assert ext.copy_values(cols, dst, threads=threads) == n
    return dst, b, x, ch


@pytest.mark.parametrize("threads", [1, 3])
def test_copy_boolean_blob_char_cpu(ext, ref, tmpfile, threads):
    """COPY ... TO 'x.fls' of BOOLEAN / BLOB / CHAR columns: the file's types
    are BOOLEAN, BLOB and VARCHAR, and the oracle decodes the values."""
    n = 70000
    dst, b, x, ch = _copy_types(ext, tmpfile, n, threads)
    rf = ref.RefFile(open(dst, "rb").read())
    assert [rf.column(c)[1] for c in range(4)] == [9, 21, 20, 4]
    got_k = np.concatenate([rf.decode(3, g) for g in range(rf.nrowgroups)]).view(np.int64)
    got_b = np.concatenate([rf.decode(0, g) for g in range(rf.nrowgroups)]).view(np.uint8)
    rows = sorted(zip(got_k.tolist(), got_b.tolist(), rf.strings_column(1), rf.strings_column(2)))
    assert rows == [(i, int(b[i]), x[i], ch[i].encode()) for i in range(n)]


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 1500, 2 * 65536 + 77])
def test_gpu_boolean_blob_decode(fl, ref, gpu, n):
    """The HIP decode of BOOLEAN (u8 FFOR / AUTO) and BLOB (FSST / DICT / AUTO)
    columns is bit-identical to the oracle, string_t records included."""
    img, cols = _table(fl, n, 7 + n)
    t, st, out = gpu_decode_all(fl, img)
    rf = ref.RefFile(img)
    for c, (name, ty, vals, _) in enumerate(cols):
        assert_column_equal(fl, rf, c, out[c], img.ptr)
        if ty == fl.BOOLEAN:
            assert np.array_equal(out[c].view(np.uint8), vals), name
        elif ty == fl.BLOB:
            assert fl.string_t_decode(out[c]) == list(vals), name


@pytest.mark.gpu
@pytest.mark.parametrize("threads", [1, 3])
def test_read_fastlanes_boolean_blob_char(ext, gpu, tmpfile, threads):
    """COPY -> read_fastlanes: BOOLEAN, BLOB and (CHAR as) VARCHAR columns come
    back with DuckDB's types and values, every row."""
    n = 70000
    dst, b, x, ch = _copy_types(ext, tmpfile, n, 1)
    names, types, rows = ext.query("read_fastlanes", dst, threads=threads)
    assert names == ["b", "x", "c", "k"] and types == ["BOOLEAN", "BLOB", "VARCHAR", "BIGINT"]
    rows.sort(key=lambda r: int(r[3]))
    assert rows == [["true" if b[i] else "false", _duck_blob(x[i]), ch[i], str(i)] for i in range(n)]


@pytest.mark.gpu
def test_filters_on_boolean_and_blob(ext, gpu, tmpfile):
    """Pushed-down comparisons on BOOLEAN (u8) and BLOB (bytes compared
    unsigned, as DuckDB's memcmp order) select the same rows as Python."""
    n = 70000
    dst, b, x, ch = _copy_types(ext, tmpfile, n)
    _, _, rows = ext.query("read_fastlanes", dst, where=[(0, "= true")])
    assert sorted(int(r[3]) for r in rows) == [i for i in range(n) if b[i]]
    probe = b"\x00\xff'\"\\"
    for op, keep in (("=", lambda v: v == probe), (">", lambda v: v > probe), ("<=", lambda v: v <= probe)):
        _, _, rows = ext.query("read_fastlanes", dst, where=[(1, f"{op} {probe.hex()}")])
        assert sorted(int(r[3]) for r in rows) == [i for i in range(n) if keep(x[i])], op
    _, _, rows = ext.query("read_fastlanes", dst, where=[(0, "= false"), (1, "= ")])
    assert sorted(int(r[3]) for r in rows) == [i for i in range(n) if not b[i] and x[i] == b""]


@pytest.mark.gpu
def test_scan_fastlanes_and_facade_render_boolean_blob(ext, gpu, tmpfile):
    """scan_fastlanes (the reference facade: its first column as VARCHAR)
    renders BOOLEAN as true/false and BLOB as DuckDB's escaped text (BLOB
    copied to the front with COPY (SELECT x, b ...)); the typed facade
    read API boxes Value::BOOLEAN / Value::BLOB."""
    n = 3000
    dst, b, x, ch = _copy_types(ext, tmpfile, n)
    # the reference's scan_fastlanes binds one VARCHAR column, "data" (the first)
    _, types, rows = ext.query("scan_fastlanes", dst)
    assert types == ["VARCHAR"] and rows == [["true" if b[i] else "false"] for i in range(n)]
    blob_first = tmpfile("blob_first.fls")
    assert ext.copy("read_fastlanes", dst, blob_first, proj=[1, 0]) == n
    _, types, rows = ext.query("scan_fastlanes", blob_first)
    assert types == ["VARCHAR"] and rows == [[_duck_blob(x[i])] for i in range(n)]
    names, ftypes, frows, _ = ext.facade_read(dst)
    assert ftypes == ["BOOLEAN", "BLOB", "VARCHAR", "BIGINT"]
    assert frows == [["true" if b[i] else "false", _duck_blob(x[i]), ch[i], str(i)] for i in range(n)]


# ---- BIT: stored as its bitstring bytes, read back as BLOB (reference
# src/type_mapping.cpp:41-42 maps LogicalTypeId::BIT to BYTE_ARRAY, and
# BYTE_ARRAY back to BLOB at :93-94) ----
def _bitstring(bits: str) -> bytes:
    """DuckDB's BIT storage (Bit::ToBit): byte 0 = padding bit count, then the
    bits most significant first, the padding bits at the top of byte 1 set"""
    pad = (8 - len(bits) % 8) % 8
    full = "1" * pad + bits
    return bytes([pad]) + int(full, 2).to_bytes(len(full) // 8, "big")


def _bits(n, rng):
    out = ["".join("01"[int(b)] for b in rng.integers(0, 2, int(k))) for k in rng.integers(1, 70, n)]
    out[0] = "1"
    if n > 1:
        out[1] = "0" * 64
    return out


def test_bitstring_helper_matches_duckdb_layout():
    assert _bitstring("1") == bytes([7, 0xFF])                     # 7 padding ones, then 1
    assert _bitstring("0") == bytes([7, 0xFE])
    assert _bitstring("01010101") == bytes([0, 0x55])
    assert _bitstring("101") == bytes([5, 0b11111101])


@pytest.mark.parametrize("threads", [1, 3])
def test_copy_bit_column_stored_as_blob_cpu(ext, ref, tmpfile, threads):
    """COPY of a BIT column: the file's column is BLOB (the writer has no BIT
    type, as the reference's FastLanes has none) holding each value's
    bitstring bytes; the oracle decodes them."""
    n = 9000
    bits = _bits(n, np.random.default_rng(11))
    dst = tmpfile("bits.fls")
    assert ext.copy_values([("v", "BIT", bits), ("k", "BIGINT", list(range(n)))], dst, threads=threads) == n
    rf = ref.RefFile(open(dst, "rb").read())
    assert [rf.column(c)[1] for c in range(2)] == [21, 4]
    got_k = np.concatenate([rf.decode(1, g) for g in range(rf.nrowgroups)]).view(np.int64)
    rows = sorted(zip(got_k.tolist(), rf.strings_column(0)))
    assert rows == [(i, _bitstring(bits[i])) for i in range(n)]


@pytest.mark.gpu
def test_read_fastlanes_bit_roundtrip_as_blob(ext, gpu, tmpfile):
    """COPY of a BIT column -> read_fastlanes on the GPU
    gives a BLOB column whose bytes are the BIT values' bitstrings, every row
    (the reference reads its BYTE_ARRAY columns back as BLOB)."""
    n = 70000
    bits = _bits(n, np.random.default_rng(12))
    dst = tmpfile("bits_gpu.fls")
    assert ext.copy_values([("v", "BIT", bits), ("k", "BIGINT", list(range(n)))], dst) == n
    names, types, rows = ext.query("read_fastlanes", dst, threads=2)
    assert names == ["v", "k"] and types == ["BLOB", "BIGINT"]
    rows.sort(key=lambda r: int(r[1]))
    assert rows == [[_duck_blob(_bitstring(bits[i])), str(i)] for i in range(n)]
