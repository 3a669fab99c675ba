"""Independent numpy restatement of the FastLanes decode path (ORACLE, test-only).

TEST INFRASTRUCTURE ONLY: imported by tests/ to cross-check oracle/flsref.c and
to generate tests/golden/ fixtures.  Never imported by the product package.

PARITY UNPINNED against upstream cwida/FastLanes bytes (the submodule named at
/root/reference/.gitmodules:9-12 is empty; no .fls fixture exists) -- see
oracle/flsref.h.  This module is written from the FastLanes paper's layout
independently of flsref.c (vectorised index arithmetic instead of loops), so the
two restatements check each other.

Layout (paper sec. 3-4; reference decode call src/fastlanes_facade.cpp:48):
  * vector = 1024 values; T-bit type -> 1024/T lanes x T rows; position
    p = row * (1024/T) + lane.
  * packed: lane L's values concatenated at W bits each into W words of T bits;
    word k of lane L lives at word index k*(1024/T) + L.
  * unified transposed layout: position p = 128a + 16b + l holds tuple
    128*FL_ORDER[b] + 16a + l, FL_ORDER = (0,4,2,6,1,5,3,7).
  * DELTA chain of lane c: tuples (c//16)*16T + c%16 + 16k, k = 0..T-1.
"""
from __future__ import annotations

import numpy as np

FL_ORDER = np.array([0, 4, 2, 6, 1, 5, 3, 7], dtype=np.int64)

ENC_FFOR, ENC_DELTA, ENC_DICT, ENC_RLE = 1, 2, 3, 4
TY_INT8, TY_INT16, TY_INT32, TY_INT64 = 1, 2, 3, 4
TY_UINT8, TY_UINT16, TY_UINT32, TY_UINT64 = 5, 6, 7, 8
TY_DATE, TY_DECIMAL, TY_VARCHAR = 10, 11, 20

_UDT = {8: np.uint8, 16: np.uint16, 32: np.uint32, 64: np.uint64}


def tau() -> np.ndarray:
    """tau[p] = original tuple index stored at transposed position p."""
    p = np.arange(1024, dtype=np.int64)
    a, b, l = p >> 7, (p >> 4) & 7, p & 15
    return 128 * FL_ORDER[b] + 16 * a + l


def _mask(w: int) -> int:
    return (1 << w) - 1


def unpack(T: int, W: int, packed: bytes) -> np.ndarray:
    """Return uint64[1024] of unsigned W-bit values in position order."""
    lanes = 1024 // T
    if W == 0:
        return np.zeros(1024, dtype=np.uint64)
    words = np.frombuffer(bytes(packed[: 128 * W]), dtype=_UDT[T]).astype(np.uint64)
    words = np.concatenate([words, np.zeros(lanes, dtype=np.uint64)])  # pad word-row
    pos = np.arange(1024, dtype=np.int64)
    row, lane = pos // lanes, pos % lanes
    bit = row * W
    k, s = bit // T, bit % T
    lo = words[k * lanes + lane]
    hi = words[(k + 1) * lanes + lane]
    # combine with python ints to avoid 64-bit shift edge cases
    out = np.empty(1024, dtype=np.uint64)
    m = _mask(W)
    for i in range(1024):
        si = int(s[i])
        v = (int(lo[i]) >> si) | ((int(hi[i]) << (T - si)) if si + W > T else 0)
        out[i] = v & m
    return out


def pack(T: int, W: int, vals: np.ndarray) -> bytes:
    """Inverse of unpack (position order in, packed bytes out)."""
    lanes = 1024 // T
    words = [0] * (lanes * (W + 1))
    m = _mask(W)
    tm = _mask(T)
    for p in range(1024):
        if W == 0:
            break
        row, lane = divmod(p, lanes)
        v = int(vals[p]) & m
        bit = row * W
        k, s = divmod(bit, T)
        words[k * lanes + lane] |= (v << s) & tm
        if s + W > T:
            words[(k + 1) * lanes + lane] |= (v >> (T - s)) & tm
    arr = np.array(words[: lanes * W], dtype=np.uint64).astype(_UDT[T])
    return arr.tobytes()


def chains(T: int) -> np.ndarray:
    """chains[c, k] = tuple index of step k of chain c."""
    c = np.arange(1024 // T, dtype=np.int64)[:, None]
    k = np.arange(T, dtype=np.int64)[None, :]
    return (c // 16) * 16 * T + (c % 16) + 16 * k


def delta_decode(T: int, u: np.ndarray, for_base: int, bases: np.ndarray) -> np.ndarray:
    """u: unpacked values in transposed position order. Returns tuple-order values mod 2^T."""
    tm = _mask(T)
    d = np.zeros(1024, dtype=object)
    t = tau()
    d[t] = [(int(x) + for_base) & tm for x in u]
    ch = chains(T)
    out = np.zeros(1024, dtype=object)
    for c in range(ch.shape[0]):
        acc = int(bases[c])
        for k in range(T):
            i = int(ch[c, k])
            acc = (acc + int(d[i])) & tm
            out[i] = acc
    return out


# --- container (independent of flsref.c's parser) ---------------------------

def _u(b, off, n):
    return int.from_bytes(bytes(b[off:off + n]), "little")


def open_image(img: bytes) -> dict:
    assert img[:8] == b"FLSAMD01" and img[-4:] == b"FLSF"
    foff, flen = _u(img, len(img) - 16, 8), _u(img, len(img) - 8, 4)
    p = foff
    assert _u(img, p, 4) == 1
    f = dict(img=img, ncols=_u(img, p + 4, 4), nrows=_u(img, p + 8, 8),
             nrowgroups=_u(img, p + 16, 4), rowgroup_size=_u(img, p + 20, 4),
             row_offset=_u(img, p + 24, 8))
    q = p + 32
    cols = []
    for _ in range(f["ncols"]):
        nl = _u(img, q + 4, 2)
        cols.append(dict(type=img[q], width=img[q + 1], scale=img[q + 2],
                         name=bytes(img[q + 6:q + 6 + nl]).decode()))
        q += 6 + nl
    rgs = []
    for _ in range(f["nrowgroups"]):
        nr = _u(img, q, 4)
        chunks = [(_u(img, q + 4 + 16 * c, 8), _u(img, q + 12 + 16 * c, 8)) for c in range(f["ncols"])]
        rgs.append(dict(nrows=nr, chunks=chunks))
        q += 4 + 16 * f["ncols"]
    f["cols"], f["rgs"] = cols, rgs
    return f


def decode_chunk(f: dict, col: int, rg: int) -> list:
    """Decode one column chunk. Ints -> list of python ints (unsigned T-bit);
    VARCHAR -> list of bytes."""
    img = f["img"]
    off, _ = f["rgs"][rg]["chunks"][col]
    ch = off
    assert _u(img, ch, 4) == 0x43534C46
    enc, T, vbits, is_str = img[ch + 4], img[ch + 5], img[ch + 6], img[ch + 7]
    nvec = _u(img, ch + 8, 4)
    meta, packed, aux = ch + _u(img, ch + 16, 8), ch + _u(img, ch + 24, 8), ch + _u(img, ch + 32, 8)
    dict_count = _u(img, ch + 48, 4)
    tm = _mask(T)
    out: list = []
    for v in range(nvec):
        m = meta + 32 * v
        poff, fb, aoff = _u(img, m, 8), _u(img, m + 8, 8), _u(img, m + 16, 8)
        vn, W, acount = _u(img, m + 24, 2), img[m + 26], _u(img, m + 28, 4)
        u = unpack(T, W, img[packed + poff: packed + poff + 128 * W])
        if enc == ENC_FFOR:
            vals = [(int(x) + fb) & tm for x in u]
        elif enc == ENC_DELTA:
            nb = 1024 // T
            bases = np.frombuffer(bytes(img[aux + aoff: aux + aoff + nb * T // 8]), dtype=_UDT[T])
            vals = list(delta_decode(T, u, fb, bases))
        elif enc == ENC_DICT:
            codes = [(int(x) + fb) & tm for x in u]
            if is_str:
                offs = np.frombuffer(bytes(img[aux: aux + 4 * (dict_count + 1)]), dtype=np.uint32)
                base = aux + 4 * (dict_count + 1)
                vals = [bytes(img[base + int(offs[c]): base + int(offs[c + 1])]) for c in codes]
            else:
                d = np.frombuffer(bytes(img[aux: aux + dict_count * vbits // 8]), dtype=_UDT[vbits])
                vals = [int(d[c]) for c in codes]
        elif enc == ENC_RLE:
            bases = np.frombuffer(bytes(img[aux + aoff: aux + aoff + 128]), dtype=np.uint16)
            idx = delta_decode(16, u, fb, bases)
            runs = np.frombuffer(bytes(img[aux + aoff + 128: aux + aoff + 128 + acount * vbits // 8]),
                                 dtype=_UDT[vbits])
            vals = [int(runs[int(i)]) for i in idx]
        else:
            raise ValueError(f"bad encoding {enc}")
        out.extend(vals[:vn])
    return out
