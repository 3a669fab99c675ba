"""The FastLanes-shaped CPU decoder (oracle/flsfast.cpp, bench.py's
cpu_baseline) decodes exactly what the oracle (oracle/flsref.c) decodes:
every encoding (FFOR / DELTA at T = 8/16/32/64, DICT int + string, RLE, ALP
float + double, FSST), every bit width, ragged tails, both builds (generic
x86-64 as the reference builds FastLanes, and AVX-512 where available).
CPU only."""
import ctypes as C

import numpy as np
import pytest

from oracle import flsfast


def _decode_fast(fl, img, build, nthreads=3):
    rf_cols = []
    from oracle import flsref
    rf = flsref.RefFile(img)
    obs = [rf.out_width(c) for c in range(rf.ncols)]
    d = flsfast.Decoder(img, img.ptr, img.len, obs, rf.nrows, 0, rf.nrowgroups, build)
    n = d.decode(nthreads)
    assert n == rf.nrows * rf.ncols
    return rf, d


def _check(fl, img, build):
    rf, d = _decode_fast(fl, img, build)
    for c in range(rf.ncols):
        name, ty = rf.column(c)[:2]
        got = d.outs[c][: rf.nrows * rf.out_width(c)]
        if ty == fl.VARCHAR:
            assert fl.string_t_decode(got) == rf.strings_column(c), name
        else:
            exp = np.concatenate([rf.decode(c, rg) for rg in range(rf.nrowgroups)])
            assert np.array_equal(got, exp), name


@pytest.mark.parametrize("build", flsfast.available())
def test_every_type_width_and_encoding(fl, build):
    rng = np.random.default_rng(11)
    n = 70000   # two row groups at 65,536 with a ragged tail vector (4464 = 4 x 1024 + 368)
    cols = []
    for ty, dt in ((fl.INT8, np.int8), (fl.INT16, np.int16), (fl.INT32, np.int32), (fl.INT64, np.int64)):
        bits = np.iinfo(dt).bits
        for w in sorted({0, 1, 3, bits // 2, bits - 1, bits}):
            hi = 1 << min(w, 62)
            v = (rng.integers(0, hi, n, dtype=np.uint64) if w else np.zeros(n, np.uint64)).astype(dt)
            cols.append((f"ffor_{bits}_{w}", ty, v, fl.ENC_FFOR))
        steps = rng.integers(0, 3, n).astype(dt)
        cols.append((f"delta_{bits}", ty, np.cumsum(steps, dtype=dt), fl.ENC_DELTA))
        cols.append((f"delta_wide_{bits}", ty, rng.integers(np.iinfo(dt).min, np.iinfo(dt).max, n, dtype=dt),
                     fl.ENC_DELTA))
    cols.append(("dict_i64", fl.INT64, rng.integers(0, 9, n) * 1000003, fl.ENC_DICT))
    cols.append(("rle_i32", fl.INT32, np.repeat(rng.integers(-5, 9, n // 37 + 1), 37)[:n].astype(np.int32),
                 fl.ENC_RLE))
    cols.append(("alp_d", fl.DOUBLE, np.where(rng.random(n) < 0.05, rng.random(n), np.round(rng.normal(0, 99, n), 2)),
                 fl.ENC_ALP))
    cols.append(("alp_f", fl.FLOAT, np.round(rng.normal(0, 50, n), 1).astype(np.float32), fl.ENC_ALP))
    words = ["AIR", "RAIL", "a longer dictionary entry", "SHIP"]
    cols.append(("dict_s", fl.VARCHAR, [words[i] for i in rng.integers(0, 4, n)], fl.ENC_DICT))
    cols.append(("fsst_s", fl.VARCHAR, [("abc" * int(k)) + chr(200 + int(k) % 50) for k in rng.integers(0, 12, n)],
                 fl.ENC_FSST))
    img = fl.write_image(cols)
    _check(fl, img, build)


@pytest.mark.parametrize("wl", ["lineitem_full", "lineitem_dbl"])
def test_lineitem_matches_oracle(fl, wl):
    img = fl.gen_image(wl, 0.02)
    for build in flsfast.available():
        _check(fl, img, build)


def test_rowgroup_subrange(fl):
    img = fl.gen_image("lineitem_full", 0.05)   # 5 row groups
    from oracle import flsref
    rf = flsref.RefFile(img)
    obs = [rf.out_width(c) for c in range(rf.ncols)]
    rows = sum(rf.rowgroup_rows(r) for r in (2, 3))
    d = flsfast.Decoder(img, img.ptr, img.len, obs, rows, 2, 4)
    assert d.decode(2) == rows * rf.ncols
    exp = np.concatenate([rf.decode(0, 2), rf.decode(0, 3)])
    assert np.array_equal(d.outs[0][: rows * 8], exp)
