"""GPU parity: the HIP decode (through the C-ABI) must be bit-identical to the
oracle (oracle/flsref.c) and to the generators' ground truth.  Integer and
byte work -> exact equality, no tolerance."""
import numpy as np
import pytest

from helpers import INT_TYPE, SIGNED, UNSIGNED, assert_column_equal, gpu_decode_all, width_sweep_values

pytestmark = pytest.mark.gpu


def _check_image(fl, ref, img, cols=None):
    t, st, out = gpu_decode_all(fl, img, cols)
    rf = ref.RefFile(img)
    for c, got in out.items():
        assert_column_equal(fl, rf, c, got, img.ptr)
    return t, st


@pytest.mark.parametrize("T", [8, 16, 32, 64])
def test_ffor_every_width(fl, ref, gpu, T):
    rng = np.random.default_rng(100 + T)
    v = width_sweep_values(T, rng)
    img = fl.write_image([("v", INT_TYPE[T], v, fl.ENC_FFOR)])
    _check_image(fl, ref, img)


@pytest.mark.parametrize("T", [8, 16, 32, 64])
def test_delta_every_width(fl, ref, gpu, T):
    rng = np.random.default_rng(200 + T)
    sweep = width_sweep_values(T, rng)            # arbitrary (unsorted) data
    keys = np.cumsum(rng.integers(0, 5, 70000)).astype(np.uint64)   # sorted keys (wrapping for small T)
    keys = keys.astype(UNSIGNED[T]).view(SIGNED[T])
    img = fl.write_image([("v", INT_TYPE[T], np.concatenate([sweep, keys]), fl.ENC_DELTA)])
    _check_image(fl, ref, img)


@pytest.mark.parametrize("T", [8, 16, 32, 64])
def test_rle_every_type(fl, ref, gpu, T):
    rng = np.random.default_rng(300 + T)
    lens = rng.integers(1, 200, 2000)
    vals = rng.integers(-(1 << (T - 1)), (1 << (T - 1)) - 1, len(lens), dtype=np.int64)
    v = np.repeat(vals, lens)[:140001].astype(SIGNED[T])
    img = fl.write_image([("r", INT_TYPE[T], v, fl.ENC_RLE)])
    _check_image(fl, ref, img)


@pytest.mark.parametrize("T", [8, 16, 32, 64])
def test_dict_int(fl, ref, gpu, T):
    rng = np.random.default_rng(400 + T)
    d = rng.integers(-(1 << (T - 1)), (1 << (T - 1)) - 1, 300, dtype=np.int64)
    v = d[rng.integers(0, len(d), 100000)].astype(SIGNED[T])
    img = fl.write_image([("d", INT_TYPE[T], v, fl.ENC_DICT)])
    _check_image(fl, ref, img)


def test_dict_strings_inline_and_pointer(fl, ref, gpu):
    rng = np.random.default_rng(5)
    words = ["", "a", "REG AIR", "exactly12chr", "thirteen chars", "DELIVER IN PERSON",
             "x" * 100] + [f"w{i:05d}-" + "y" * (i % 20) for i in range(1500)]
    v = [words[i] for i in rng.integers(0, len(words), 150000)]
    img = fl.write_image([("s", fl.VARCHAR, v, fl.ENC_DICT)])
    t, _ = _check_image(fl, ref, img)
    got = fl.string_t_decode(t.device_copy_out(0, 0, 5000))
    assert got == [x.encode() for x in v[:5000]]


@pytest.mark.parametrize("n", [1, 5, 1023, 1024, 1025, 65535, 65536, 65537, 3 * 65536 + 777])
def test_ragged_sizes(fl, ref, gpu, n):
    rng = np.random.default_rng(n)
    a = rng.integers(-50, 50, n).astype(np.int32)
    b = np.cumsum(rng.integers(0, 4, n)).astype(np.int64)
    s = [["N", "O", "DELIVER IN PERSON"][i] for i in rng.integers(0, 3, n)]
    img = fl.write_image([("a", fl.INT32, a, fl.ENC_FFOR), ("b", fl.INT64, b, fl.ENC_DELTA),
                          ("s", fl.VARCHAR, s, fl.ENC_DICT), ("r", fl.INT16, (b // 100).astype(np.int16), fl.ENC_RLE)])
    _check_image(fl, ref, img)


def test_auto_encoding_mix(fl, ref, gpu):
    rng = np.random.default_rng(11)
    n = 200000
    cols = [("ffor", fl.INT64, rng.integers(0, 1 << 40, n), fl.ENC_AUTO),
            ("sorted", fl.INT64, np.cumsum(rng.integers(0, 3, n)), fl.ENC_AUTO),
            ("runs", fl.INT32, np.repeat(rng.integers(0, 1000, n // 500), 500), fl.ENC_AUTO),
            ("lowcard", fl.UINT16, rng.integers(0, 7, n) * 1000, fl.ENC_AUTO),
            ("date", fl.DATE, 8035 + rng.integers(0, 2500, n), fl.ENC_AUTO),
            ("dec", fl.DECIMAL, rng.integers(0, 10**9, n), fl.ENC_AUTO, 15, 2)]
    img = fl.write_image(cols)
    _check_image(fl, ref, img)


def test_column_projection(fl, ref, gpu):
    img = fl.gen_image("lineitem", 0.01)
    _check_image(fl, ref, img, cols=[0, 5, 13])


@pytest.mark.parametrize("scale", [0.01, 0.1])
def test_lineitem_vs_oracle_and_generator(fl, ref, gpu, scale):
    img = fl.gen_image("lineitem", scale)
    t, st = _check_image(fl, ref, img)
    n = t.nrows
    assert st.values == n * 15
    # and against the generator's ground truth directly
    for c in range(15):
        name, ty, _, _, ob = t.schema()[c]
        got = t.device_copy_out(c)
        if ty == fl.VARCHAR:
            codes = fl.gen_values("lineitem", c, 0, n, np.uint32, scale)
            strs = fl.string_t_decode(got[: 16 * 2000])
            exp = [fl.gen_dict_string("lineitem", c, int(k)).encode() for k in codes[:2000]]
            assert strs == exp, name
        else:
            exp = fl.gen_values("lineitem", c, 0, n, fl.NP_DTYPE[ty], scale)
            assert np.array_equal(got.view(fl.NP_DTYPE[ty]), exp), name


def test_c1_file_roundtrip(fl, ref, gpu, tmpfile):
    img = fl.gen_image("c1")
    path = tmpfile("c1.fls")
    img.write(path)
    conn = fl.Connection()
    t = conn.read_fls(path)
    assert t.nrows == 1_000_000 and t.nrowgroups == 16 and t.rowgroup_rows(15) == 16960
    t.device_upload()
    t.device_decode()
    t.device_sync()
    got = t.device_copy_out(0).view(np.int32)
    exp = fl.gen_values("c1", 0, 0, 1_000_000, np.int32)
    assert np.array_equal(got, exp)
    assert got.min() >= 1_000_000 and got.max() < 1_000_128


def test_repeated_decode_is_idempotent(fl, ref, gpu):
    img = fl.gen_image("lineitem", 0.01)
    conn = fl.Connection()
    t = conn.read_image(img)
    t.device_upload()
    t.device_decode()
    t.device_sync()
    first = [t.device_copy_out(c) for c in range(t.ncols)]
    for _ in range(3):
        t.device_decode()
    st = t.device_sync()
    assert st.launches == 4 and st.kernel_ms > 0
    for c in range(t.ncols):
        assert np.array_equal(t.device_copy_out(c), first[c])


def test_scan_and_materialize_match_oracle(fl, ref, gpu):
    img = fl.gen_image("lineitem", 0.1)   # 10 row groups
    rf = ref.RefFile(img)
    conn = fl.Connection()
    t = conn.read_image(img)
    seen = 0
    for first_row, cols in t.scan(cols=[0, 1, 8, 10]):
        rg = first_row // 65536
        for c in (0, 1, 10):
            assert np.array_equal(cols[c], rf.decode(c, rg)), (rg, c)
        assert cols[2] is None
        assert fl.string_t_decode(cols[8][:16 * 64]) == rf.strings(rf.decode(8, rg))[:64]
        seen += 1
    assert seen == rf.nrowgroups
    first_row, cols = t.materialize(3)
    assert first_row == 3 * 65536
    for c in range(15):
        if rf.column(c)[1] != 20:
            assert np.array_equal(cols[c], rf.decode(c, 3)), c


def test_scan_batches_and_subrange(fl, ref, gpu, monkeypatch):
    monkeypatch.setenv("FLS_SCAN_BATCH", "3")
    img = fl.gen_image("c3", nrows=20 * 65536 + 5)
    rf = ref.RefFile(img)
    conn = fl.Connection()
    t = conn.read_image(img)
    got = list(t.scan(rg_begin=4, rg_end=21))
    assert [r // 65536 for r, _ in got] == list(range(4, 21))
    for r, cols in got:
        assert np.array_equal(cols[0], rf.decode(0, r // 65536))


def test_corrupt_dictionary_code_is_reported(fl, ref, gpu):
    v = np.arange(5000) % 7
    img = fl.write_image([("d", fl.INT32, v, fl.ENC_DICT)])
    raw = bytearray(img.tobytes())
    rf = ref.RefFile(bytes(raw))
    # shrink dict_count in the first chunk header (offset 256 + 48) -> codes out of range
    import struct
    assert struct.unpack_from("<I", raw, 256)[0] == 0x43534C46
    struct.pack_into("<I", raw, 256 + 48, 3)
    conn = fl.Connection()
    t = conn.read_image(bytes(raw))
    t.device_upload()
    t.device_decode()
    with pytest.raises(fl.FlsError, match="corrupt"):
        t.device_sync()
    del rf


def test_scan_sharded_over_two_device_slots(fl, ref, gpu, monkeypatch):
    """The in-process multi-GPU scan path (one stream + two-slot pipeline per
    device, contiguous row-group ranges, in-order delivery) exercised with the
    same GPU listed twice."""
    monkeypatch.setenv("FLS_SCAN_BATCH", "2")
    img = fl.gen_image("lineitem", 0.1)
    rf = ref.RefFile(img)
    conn = fl.Connection([0, 0])
    t = conn.read_image(img)
    got = list(t.scan(cols=[0, 5, 14]))
    assert [r // 65536 for r, _ in got] == list(range(rf.nrowgroups))
    for first, cols in got:
        rg = first // 65536
        assert np.array_equal(cols[0], rf.decode(0, rg)) and np.array_equal(cols[5], rf.decode(5, rg))
    # materialize picks the owning device of the row group
    first, cols = t.materialize(rf.nrowgroups - 1, cols=[0])
    assert np.array_equal(cols[0], rf.decode(0, rf.nrowgroups - 1))


@pytest.mark.parametrize("rgsz", [1024, 8192])
def test_small_rowgroups_decode_and_scan(fl, ref, gpu, monkeypatch, rgsz):
    """Files written with ROW_GROUP_SIZE < 65536 (COPY option): device decode
    and the batched scan place row group r at first_row = r * rgsz."""
    monkeypatch.setenv("FLS_SCAN_BATCH", "3")
    rng = np.random.default_rng(rgsz)
    n = 7 * rgsz + 333
    a = rng.integers(-(1 << 40), 1 << 40, n)
    b = np.cumsum(rng.integers(0, 9, n)).astype(np.int32)
    s = [["AIR", "MAIL", "TRUCK", "REG AIR LONGER THAN TWELVE"][i] for i in rng.integers(0, 4, n)]
    img = fl.write_image([("a", fl.INT64, a, fl.ENC_FFOR), ("b", fl.INT32, b, fl.ENC_DELTA),
                          ("s", fl.VARCHAR, s, fl.ENC_DICT)], rowgroup=rgsz)
    rf = ref.RefFile(img)
    t, _ = _check_image(fl, ref, img)
    got = list(t.scan())
    assert [r for r, _ in got] == [g * rgsz for g in range(8)]
    for first, cols in got:
        g = first // rgsz
        assert np.array_equal(cols[0], rf.decode(0, g)) and np.array_equal(cols[1], rf.decode(1, g))
        assert fl.string_t_decode(cols[2]) == rf.strings(rf.decode(2, g))


# Work distribution policies (FLS_DECODE_POLICY, read per decode call): the
# default (0: small launches like this one take the balanced split), the work
# queue of whole chunks (64), static grid-stride (1), the balanced split of
# vector ranges (32: a chunk may be cut between waves, including inside the
# ragged last row group) with and without dynamic tail pieces, and the guided
# queue (64 + FLS_GUIDED_MIN_VECS: whole chunks, then ever smaller pieces,
# cut inside chunks and the ragged last row group).  Every policy must decode
# identically.
@pytest.mark.parametrize("env", [
    {"FLS_DECODE_POLICY": "0"},
    {"FLS_DECODE_POLICY": "64"},
    {"FLS_DECODE_POLICY": "1"},
    {"FLS_DECODE_POLICY": "32"},
    {"FLS_DECODE_POLICY": "32", "FLS_STATIC_PCT": "70", "FLS_TAIL_PIECES": "3"},
    {"FLS_DECODE_POLICY": "32", "FLS_STATIC_PCT": "0", "FLS_TAIL_PIECES": "1"},
    {"FLS_DECODE_POLICY": "32", "FLS_BLOCKS_PER_CU": "1"},
    {"FLS_DECODE_POLICY": "64", "FLS_GUIDED_MIN_VECS": "0"},
    {"FLS_DECODE_POLICY": "64", "FLS_GUIDED_MIN_VECS": "1", "FLS_GUIDED_FACTOR": "8"},
    {"FLS_DECODE_POLICY": "64", "FLS_GUIDED_MIN_VECS": "8", "FLS_GUIDED_FACTOR": "1"},
    {"FLS_DECODE_POLICY": "64", "FLS_GUIDED_MIN_VECS": "3", "FLS_GUIDED_FACTOR": "2", "FLS_BLOCKS_PER_CU": "1"},
], ids=["default", "queue", "static", "balanced", "balanced_tail70", "tail_only", "balanced_1blk", "queue_chunks",
        "guided_1", "guided_8", "guided_3_1blk"])
def test_work_distribution_policies(fl, ref, gpu, monkeypatch, env):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(77)
    n = 5 * 65536 + 1234
    a = rng.integers(-50, 50, n).astype(np.int32)
    b = np.cumsum(rng.integers(0, 4, n)).astype(np.int64)
    s = [["N", "O", "DELIVER IN PERSON"][i] for i in rng.integers(0, 3, n)]
    r = (b // 100).astype(np.int16)
    img = fl.write_image([("a", fl.INT32, a, fl.ENC_FFOR), ("b", fl.INT64, b, fl.ENC_DELTA),
                          ("s", fl.VARCHAR, s, fl.ENC_DICT), ("r", fl.INT16, r, fl.ENC_RLE),
                          ("d", fl.INT32, (a % 7).astype(np.int32), fl.ENC_DICT)])
    _check_image(fl, ref, img)
    _check_image(fl, ref, img, [1, 2])
