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


def assert_strings_equal(fl, rf, c: int, got: np.ndarray, row0: int = 0):
    """string_t records vs the oracle's strings (any string encoding): lengths,
    contents through the pointers, zero padding of inline records, prefixes."""
    exp = rf.strings_column(c)[row0:row0 + len(got) // 16]
    rec = got.reshape(-1, 16)
    assert fl.string_t_decode(got) == exp
    for i in range(0, len(exp), max(1, len(exp) // 4096)):
        e = exp[i]
        if len(e) <= 12:
            assert bytes(rec[i, 4:16]) == e + b"\0" * (12 - len(e)), i
        else:
            assert bytes(rec[i, 4:8]) == e[:4], i


def assert_column_equal(fl, rf, c: int, got: np.ndarray, base_ptr: int):
    name, ty, _, _ = rf.column(c)
    try:
        exp = rf.decode_column(c, nthreads=8)
    except ValueError:              # FSST: strings are not inside the image
        assert ty in (20, 21)
        assert_strings_equal(fl, rf, c, got)
        return
    if ty in (20, 21):
        exp = expected_string_t(rf, exp, base_ptr)
    assert got.shape == exp.shape, (name, got.shape, exp.shape)
    if not np.array_equal(got, exp):
        w = 16 if ty in (20, 21) else rf.out_width(c)
        bad = np.nonzero((got.reshape(-1, w) != exp.reshape(-1, w)).any(axis=1))[0]
        raise AssertionError(f"column {name}: {len(bad)} mismatching rows, first {bad[:8]}")


WORDS = ("furiously carefully quickly slyly blithely ironic final regular express pending special bold even "
         "silent unusual deposits requests accounts packages instructions foxes ideas theodolites pinto beans "
         "platelets asymptotes dependencies courts dolphins multipliers sauternes warthogs frets dinos attainments "
         "somas sentiments the of and to above across after against along among around at about according "
         "sleep wake are cajole haggle nag use boost affix detect integrate maintain nod was").split()


def fsst_text(n, rng):
    """TPC-H-comment-like strings (10..43 chars cut from word text)."""
    out = []
    for _ in range(n):
        k = int(rng.integers(10, 44))
        words = [WORDS[j] for j in rng.integers(0, len(WORDS), 12)]
        out.append(" ".join(words)[:k])
    return out


def special_doubles(n, rng):
    pool = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, -5e-324, 1.7976931348623157e308,
                     2.2250738585072014e-308, 1e300, 0.1, 1 / 3])
    return pool[rng.integers(0, len(pool), n)]


# ---- pushed-down filters: numpy restatement of DuckDB comparison semantics ----
def _cmp(a, v):
    """-1/0/1 of a (numpy column or list of bytes) against constant v, with
    DuckDB's float order (NaN == NaN, NaN above every number, -0 == 0)."""
    if isinstance(a, list):
        return np.array([(x > v) - (x < v) for x in a], dtype=np.int8)
    if a.dtype.kind == "f":
        v = np.float64(v)
        an = np.isnan(a)
        if np.isnan(v):
            return np.where(an, 0, -1).astype(np.int8)
        a64 = a.astype(np.float64)
        c = (a64 > v).astype(np.int8) - (a64 < v).astype(np.int8)
        return np.where(an, 1, c).astype(np.int8)
    # integers: exact (object arithmetic for 64-bit unsigned / mixed signs)
    a = a.astype(np.int64) if a.dtype.kind == "i" else a.astype(np.uint64)
    if a.dtype == np.uint64 and v < 0:
        return np.ones(len(a), np.int8)
    vv = a.dtype.type(v)
    return (a > vv).astype(np.int8) - (a < vv).astype(np.int8)


def filter_mask(cols: dict, terms, n: int) -> np.ndarray:
    """Rows satisfying the conjunction of clauses; terms = (col, op, value[, clause])
    as in Table.scan_filtered.  cols[c] = numpy values or list of bytes."""
    ops = {"=": lambda c: c == 0, "!=": lambda c: c != 0, "<": lambda c: c < 0, "<=": lambda c: c <= 0,
           ">": lambda c: c > 0, ">=": lambda c: c >= 0}
    clauses = {}
    for i, t in enumerate(terms):
        clauses.setdefault(t[3] if len(t) > 3 else 1000000 + i, []).append(t)
    out = np.ones(n, dtype=bool)
    for cl in clauses.values():
        acc = np.zeros(n, dtype=bool)
        for col, op, val, *_ in cl:
            if op == "is_null":
                continue
            if op == "is_not_null":
                acc[:] = True
                continue
            v = val.encode() if isinstance(val, str) else val
            acc |= ops[op](_cmp(cols[col], v))
        out &= acc
    return out
