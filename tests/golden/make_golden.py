"""Regenerate tests/golden/*.npz (committed fixtures).

* pack_T{T}_W{W}.npz -- bit-packing known answers produced by the independent
  numpy restatement (oracle/flsref_np.py): values in position order + packed
  bytes in the FastLanes interleaved layout.
* img_*.npz -- small .fls images written by the product writer from seeded
  inputs, with the inputs themselves as the expected decode (integer codecs
  are lossless, so the input IS the ground truth).

No reference fixture exists for this path (the reference's only data file,
third_party/fastlanes/data/fls/data.fls, lives in an empty submodule), so these
pin our restatement against itself across changes; parity with upstream
FastLanes bytes stays unpinned.
Run: python tests/golden/make_golden.py
"""
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT))

import pkgload  # noqa: E402
from oracle import flsref_np  # noqa: E402


def main():
    fl = pkgload.load()
    rng = np.random.default_rng(20250824)
    for T, W in [(8, 0), (8, 3), (8, 8), (16, 5), (16, 16), (32, 1), (32, 7), (32, 31), (32, 32),
                 (64, 5), (64, 33), (64, 64)]:
        m = (1 << W) - 1
        vals = np.array([int.from_bytes(rng.bytes(8), "little") & m for _ in range(1024)], dtype=np.uint64)
        packed = np.frombuffer(flsref_np.pack(T, W, vals), dtype=np.uint8)
        assert np.array_equal(flsref_np.unpack(T, W, packed.tobytes()), vals)
        np.savez_compressed(HERE / f"pack_T{T}_W{W}.npz", T=T, W=W, values=vals, packed=packed)

    n = 2500  # 2 full vectors + a 452-value tail
    cases = {
        "ffor_i32": [("v", fl.INT32, (1000000 + rng.integers(0, 128, n)).astype(np.int32), fl.ENC_FFOR)],
        "delta_i64": [("k", fl.INT64, np.cumsum(rng.integers(0, 30, n)).astype(np.int64) + 7, fl.ENC_DELTA)],
        "delta_i16_signed": [("k", fl.INT16, rng.integers(-3000, 3000, n).astype(np.int16), fl.ENC_DELTA)],
        "dict_i8": [("d", fl.INT8, rng.integers(-5, 5, n).astype(np.int8), fl.ENC_DICT)],
        "rle_i32": [("r", fl.INT32, np.repeat(rng.integers(-9, 9, n // 25 + 1), 25)[:n].astype(np.int32), fl.ENC_RLE)],
        "dict_str": [("s", fl.VARCHAR, [["REG AIR", "DELIVER IN PERSON", "", "x"][i] for i in rng.integers(0, 4, n)],
                      fl.ENC_DICT)],
    }
    for name, cols in cases.items():
        img = fl.write_image(cols)
        payload = {"image": np.frombuffer(img.tobytes(), dtype=np.uint8)}
        for c, (_, ty, vals, _) in enumerate(cols):
            payload[f"col{c}"] = np.array(vals, dtype="S") if ty == fl.VARCHAR else np.asarray(vals)
        np.savez_compressed(HERE / f"img_{name}.npz", **payload)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
