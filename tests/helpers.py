"""Shared test helpers: build columns that hit every (T, W) combination, decode
on the GPU, and compare bit-exactly with the oracle (oracle/flsref.c)."""
from __future__ import annotations

import numpy as np

TBITS = {1: 8, 2: 16, 3: 32, 4: 64, 5: 8, 6: 16, 7: 32, 8: 64, 10: 32, 11: 64}
SIGNED = {8: np.int8, 16: np.int16, 32: np.int32, 64: np.int64}
UNSIGNED = {8: np.uint8, 16: np.uint16, 32: np.uint32, 64: np.uint64}
INT_TYPE = {8: 1, 16: 2, 32: 3, 64: 4}


def width_sweep_values(T: int, rng, tail: int = 333) -> np.ndarray:
    """One 1024-value vector per bit width 0..T (FFOR residual exactly W bits),
    alternating negative / positive bases, plus a partial tail vector."""
    out = []
    tm = np.uint64((1 << T) - 1) if T < 64 else np.uint64(0xFFFFFFFFFFFFFFFF)
    for W in range(T + 1):
        wm = np.uint64((1 << W) - 1) if W < 64 else np.uint64(0xFFFFFFFFFFFFFFFF)
        r = rand64(rng, 1024) & wm
        r[rng.integers(0, 1024)] = wm
        r[rng.integers(0, 1024)] = np.uint64(0)
        # base keeps base + r inside the signed T-bit range, so the writer's FOR
        # base is exactly `base` and the residual width is exactly W
        lo, hi = -(1 << (T - 1)), (1 << (T - 1)) - (1 << W)
        base = int(rng.integers(lo, hi + 1)) if hi > lo else lo
        v = (np.uint64(base & 0xFFFFFFFFFFFFFFFF) + r) & tm
        out.append(v)
    out.append(rand64(rng, tail) & tm)
    u = np.concatenate(out)
    return u.astype(UNSIGNED[T]).view(SIGNED[T])


def rand64(rng, n: int) -> np.ndarray:
    return (rng.integers(0, 1 << 32, n, dtype=np.uint64) << np.uint64(32)) | \
        rng.integers(0, 1 << 32, n, dtype=np.uint64)


def gpu_decode_all(fl, img, cols=None):
    conn = fl.Connection()
    t = conn.read_image(img)
    t.device_upload()
    t.device_decode(cols)
    st = t.device_sync()
    sel = range(t.ncols) if cols is None else cols
    out = {c: t.device_copy_out(c) for c in sel}
    return t, st, out


def expected_string_t(rf, raw_pairs: np.ndarray, base_ptr: int) -> np.ndarray:
    """DuckDB string_t records the GPU must produce for oracle (offset, len)
    pairs, with >12-byte strings pointing into the image at base_ptr."""
    pairs = raw_pairs.view(np.uint64).reshape(-1, 2)
    n = len(pairs)
    rec = np.zeros((n, 16), dtype=np.uint8)
    rec[:, :4] = pairs[:, 1].astype(np.uint32).view(np.uint8).reshape(n, 4)
    img = np.ctypeslib.as_array((np.ctypeslib.ctypes.c_uint8 * rf.f.len).from_address(rf.base))
    offs, lens = pairs[:, 0].astype(np.int64), pairs[:, 1].astype(np.int64)
    short = lens <= 12
    for j in range(12):
        m = short & (lens > j)
        rec[m, 4 + j] = img[offs[m] + j]
    lm = ~short
    for j in range(4):
        rec[lm, 4 + j] = img[offs[lm] + j]
    rec[lm, 8:16] = (np.uint64(base_ptr) + offs[lm].astype(np.uint64)).view(np.uint8).reshape(-1, 8)
    return rec.reshape(-1)


def assert_column_equal(fl, rf, c: int, got: np.ndarray, base_ptr: int):
    exp = rf.decode_column(c, nthreads=8)
    name, ty, _, _ = rf.column(c)
    if ty == 20:
        exp = expected_string_t(rf, exp, base_ptr)
    assert got.shape == exp.shape, (name, got.shape, exp.shape)
    if not np.array_equal(got, exp):
        w = 16 if ty == 20 else rf.out_width(c)
        bad = np.nonzero((got.reshape(-1, w) != exp.reshape(-1, w)).any(axis=1))[0]
        raise AssertionError(f"column {name}: {len(bad)} mismatching rows, first {bad[:8]}")
