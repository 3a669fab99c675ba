"""Randomised parity sweep: tables of random shape -- column types, encodings,
value distributions, row counts and row-group sizes drawn from fixed seeds --
written by the CPU writer and by the writer with the GPU encoder (bytes must
agree), then decoded on the GPU and compared with the oracle
(oracle/flsref.c) column by column.  Complements the targeted tests, which
each pin one path (test_gpu_decode.py, test_alp_fsst.py, test_encode.py)."""
import numpy as np
import pytest

from helpers import assert_column_equal, gpu_decode_all

INT_TYPES = ["INT8", "INT16", "INT32", "INT64", "UINT8", "UINT16", "UINT32", "UINT64", "DATE", "DECIMAL"]
WORDS = [b"FastLanes", b"x", b"", b"carefully final deposits", b"\xff\xfe escape bytes \x00", b"a" * 40, b"REG AIR"]


def _int_values(fl, ty, n, rng):
    dt = np.dtype(fl.NP_DTYPE[ty])
    info = np.iinfo(dt)
    shape = rng.integers(0, 6)
    if shape == 0:   # full range
        return rng.integers(info.min, info.max, n, dtype=dt, endpoint=True)
    if shape == 1:   # narrow band around a random base
        base = int(rng.integers(info.min // 2, info.max // 2))
        return (base + rng.integers(0, 1 << int(rng.integers(0, 9)), n)).astype(dt)
    if shape == 2:   # sorted keys
        return np.sort(rng.integers(info.min // 4, info.max // 4, n, dtype=dt))
    if shape == 3:   # runs
        k = int(rng.integers(1, 300))
        return np.repeat(rng.integers(info.min, info.max, n // k + 1, dtype=dt, endpoint=True), k)[:n]
    if shape == 4:   # few distinct values
        return rng.integers(info.min, info.max, 5, dtype=dt, endpoint=True)[rng.integers(0, 5, n)]
    return np.full(n, int(rng.integers(info.min, info.max, dtype=dt, endpoint=True)), dtype=dt)


def _random_table(fl, seed):
    rng = np.random.default_rng(seed)
    n = int(rng.choice([1, 7, 1023, 1025, 4096, 65537, int(rng.integers(1, 200000))]))
    rowgroup = int(rng.choice([1024, 4096, 65536]))
    cols = []
    for j in range(int(rng.integers(1, 9))):
        kind = rng.integers(0, 10)
        if kind < 7:
            ty = getattr(fl, INT_TYPES[int(rng.integers(0, len(INT_TYPES)))])
            enc = [fl.ENC_AUTO, fl.ENC_FFOR, fl.ENC_DELTA, fl.ENC_DICT, fl.ENC_RLE][int(rng.integers(0, 5))]
            col = (f"i{j}", ty, _int_values(fl, ty, n, rng), enc)
            if ty == fl.DECIMAL:
                col = col + (15, 2)
            cols.append(col)
        elif kind < 8:
            ty = fl.DOUBLE if rng.integers(0, 2) else fl.FLOAT
            dt = np.float64 if ty == fl.DOUBLE else np.float32
            vals = (np.round(rng.normal(0, 1e4, n), int(rng.integers(0, 4)))).astype(dt)
            vals[rng.integers(0, n, max(1, n // 100))] = dt(np.pi)  # ALP exceptions
            cols.append((f"f{j}", ty, vals, fl.ENC_AUTO))
        else:
            enc = [fl.ENC_AUTO, fl.ENC_DICT, fl.ENC_FSST][int(rng.integers(0, 3))]
            picks = rng.integers(0, len(WORDS), n)
            vals = [WORDS[p] + (b"%d" % i if rng.integers(0, 2) and enc != fl.ENC_DICT else b"") for i, p in
                    enumerate(picks)]
            cols.append((f"s{j}", fl.VARCHAR, vals, enc))
    return cols, rowgroup


@pytest.mark.parametrize("seed", list(range(32)))
def test_random_tables_cpu_writer_decodes(fl, ref, seed):
    """CPU side: every random table is written and the oracle reads it back."""
    cols, rowgroup = _random_table(fl, seed)
    img = fl.write_image(cols, rowgroup=rowgroup)
    rf = ref.RefFile(img)
    assert rf.nrows == len(cols[0][2]) and rf.ncols == len(cols)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", list(range(32)))
def test_random_tables_gpu(fl, ref, gpu, seed):
    cols, rowgroup = _random_table(fl, seed)
    img = fl.write_image(cols, rowgroup=rowgroup)
    assert fl.write_image(cols, rowgroup=rowgroup, device=0).tobytes() == img.tobytes()
    t, st, out = gpu_decode_all(fl, img)
    rf = ref.RefFile(img)
    for c, got in out.items():
        assert_column_equal(fl, rf, c, got, img.ptr)
