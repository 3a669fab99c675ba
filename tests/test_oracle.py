"""Oracle checks (CPU): the C restatement (oracle/flsref.c) against hand-computed
known-answer tests, the independent numpy restatement (oracle/flsref_np.py) and
the committed golden fixtures (tests/golden/).  Parity with upstream FastLanes
bytes is unpinned (no fixture exists in the reference)."""
import numpy as np
import pytest

from oracle import flsref_np


def test_tau_is_bijection(ref):
    t = [ref.tau(p) for p in range(1024)]
    assert sorted(t) == list(range(1024))
    assert list(flsref_np.tau()) == t
    # FL_ORDER 0,4,2,6,1,5,3,7 on the 16-value blocks of each 128-tuple row
    assert [ref.tau(16 * b) for b in range(8)] == [128 * o for o in (0, 4, 2, 6, 1, 5, 3, 7)]
    assert ref.tau(128) == 16 and ref.tau(1) == 1


def test_kat_pack_t32_w7(ref):
    # value at position p = row*32 + lane is p mod 128 (7 bits)
    vals = np.arange(1024, dtype=np.uint64) % 128
    packed = np.frombuffer(ref.pack(32, 7, vals), dtype=np.uint32)
    assert packed.size == 7 * 32
    # lane 0: rows 0..3 hold 0,32,64,96 in bits 0..27, row 4 (value 0) straddles
    assert packed[0] == (32 << 7) | (64 << 14) | (96 << 21)
    # lane 1, word 0: rows 0..3 = 1,33,65,97 ; row 4 = 1 -> low 4 bits at 28..31
    assert packed[1] == 1 | (33 << 7) | (65 << 14) | (97 << 21) | (1 << 28)
    # word 1 of lane 1 starts with the 3 high bits of row 4's value (1 >> 4 = 0)
    # followed by row 5 (value 33) at bit 3
    assert packed[32 + 1] & 0x3FF == (33 << 3)
    assert np.array_equal(ref.unpack(32, 7, packed.tobytes()), vals)


def test_kat_pack_t64_w64_identity(ref):
    vals = np.arange(1024, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    packed = ref.pack(64, 64, vals)
    # W == T: word k of lane L is just the value at row k, i.e. identity layout
    assert np.array_equal(np.frombuffer(packed, dtype=np.uint64), vals)


@pytest.mark.parametrize("T", [8, 16, 32, 64])
def test_pack_unpack_c_vs_numpy(ref, T):
    rng = np.random.default_rng(T)
    for W in sorted({0, 1, 2, 3, T // 2 - 1, T // 2, T - 1, T} | set(rng.integers(1, T, 3).tolist())):
        W = int(W)
        hi = (1 << W) - 1
        vals = np.array([int(x) & hi for x in rng.integers(0, 1 << 62, 1024, dtype=np.uint64)], dtype=np.uint64) \
            if W < 62 else np.array([int.from_bytes(rng.bytes(8), "little") & hi for _ in range(1024)], dtype=np.uint64)
        pc = ref.pack(T, W, vals)
        pn = flsref_np.pack(T, W, vals)
        assert pc == pn, (T, W)
        assert np.array_equal(ref.unpack(T, W, pc), vals)
        assert np.array_equal(flsref_np.unpack(T, W, pn), vals)


@pytest.mark.parametrize("T", [8, 16, 32, 64])
def test_delta_chain_layout(T):
    # every lane's T rows hold one chain: stride 16 inside a block of 16*T tuples
    tau = flsref_np.tau()
    lanes = 1024 // T
    ch = flsref_np.chains(T)
    chain_of = {}
    for c in range(ch.shape[0]):
        for k in range(T):
            chain_of[int(ch[c, k])] = c
    for lane in range(lanes):
        cs = {chain_of[int(tau[row * lanes + lane])] for row in range(T)}
        assert len(cs) == 1, (T, lane, cs)


def test_golden_fixtures(ref):
    import glob
    import os
    files = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz")))
    assert files, "tests/golden fixtures missing (run tests/golden/make_golden.py)"
    checked = 0
    for f in files:
        z = np.load(f, allow_pickle=False)
        if "packed" in z:  # bit-packing KAT
            T, W = int(z["T"]), int(z["W"])
            assert np.array_equal(ref.unpack(T, W, z["packed"].tobytes()), z["values"]), f
            assert ref.pack(T, W, z["values"]) == z["packed"].tobytes(), f
        else:  # .fls image + expected decode per column
            rf = ref.RefFile(z["image"].tobytes())
            for c in range(rf.ncols):
                exp = z[f"col{c}"]
                raw = np.concatenate([rf.decode(c, rg) for rg in range(rf.nrowgroups)])
                if exp.dtype.kind == "U" or exp.dtype.kind == "S":
                    assert rf.strings(raw) == [bytes(x) if isinstance(x, bytes) else x.encode() for x in exp]
                else:
                    assert np.array_equal(raw.view(exp.dtype), exp), (f, c)
        checked += 1
    assert checked >= 8


def test_numpy_restatement_decodes_container(fl, ref):
    rng = np.random.default_rng(7)
    n = 3000
    a = np.cumsum(rng.integers(-3, 9, n)).astype(np.int64)
    b = np.repeat(rng.integers(0, 9, n // 10 + 1), 10)[:n].astype(np.int32)
    img = fl.write_image([("a", fl.INT64, a, fl.ENC_DELTA), ("b", fl.INT32, b, fl.ENC_RLE),
                          ("c", fl.INT16, (a % 300).astype(np.int16), fl.ENC_DICT)])
    f = flsref_np.open_image(img.tobytes())
    rf = ref.RefFile(img)
    for c, dt in [(0, np.uint64), (1, np.uint32), (2, np.uint16)]:
        got_np = np.array(flsref_np.decode_chunk(f, c, 0), dtype=np.uint64).astype(dt)
        assert np.array_equal(got_np, rf.decode(c, 0).view(dt))


@pytest.mark.parametrize("T", [8, 16, 32, 64])
def test_survey_layout_statements(ref, T):
    """SURVEY.md section 5's statements of the FastLanes layout, checked
    mechanically against the C restatement:
      * interleaved packing (every T), bit by bit: the W-bit value at (row r,
        lane l) starts in packed word floor(r W / T) * (1024 / T) + l at bit
        (r W) mod T and straddles into the next word of the same lane;
      * unified transposed order (T = 64): SURVEY's index(r, l) =
        FL_ORDER[r / 8] * 16 + (r % 8) * 128 + l puts in lane l exactly the
        tuples this restatement does (the delta chain l + 16 k, base tuple l),
        but in another row order: SURVEY's row r is this layout's row
        8 FL_ORDER[r / 8] + FL_ORDER[r % 8] of the same lane.  That fixed row
        permutation is the one layout fact an upstream fixture would decide
        (oracle/flsref.h, "Upstream facts")."""
    lanes = 1024 // T
    rng = np.random.default_rng(100 + T)
    for W in sorted({1, 3, T // 2 + 1, T - 1, T}):
        vals = np.array([int.from_bytes(rng.bytes(8), "little") & ((1 << W) - 1) for _ in range(1024)],
                        dtype=np.uint64)
        words = np.frombuffer(ref.pack(T, W, vals), dtype=f"<u{T // 8}")
        assert words.size == W * lanes
        for p in rng.integers(0, 1024, 64):
            r, l = divmod(int(p), lanes)
            k, b = divmod(r * W, T)
            lo = int(words[k * lanes + l]) >> b
            if b + W > T:
                lo |= int(words[(k + 1) * lanes + l]) << (T - b)
            assert lo & ((1 << W) - 1) == int(vals[p]), (T, W, r, l)
    if T == 64:
        order = (0, 4, 2, 6, 1, 5, 3, 7)
        for l in range(16):
            survey = [order[r // 8] * 16 + (r % 8) * 128 + l for r in range(64)]
            ours = [ref.tau(r * 16 + l) for r in range(64)]
            assert sorted(survey) == sorted(ours) == [l + 16 * k for k in range(64)]
            for r in range(64):
                assert survey[r] == ours[8 * order[r // 8] + order[r % 8]]
