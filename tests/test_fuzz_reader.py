"""Host-side sanitizer run: mutation fuzzing of the .fls reader
(csrc/fls_reader.hpp parse_file + everything the host reads after it) built
with g++ -fsanitize=address,undefined (tests/fuzz/fuzz_reader.cpp).

parse_file stands between an untrusted file and the decode kernels; an
out-of-bounds offset it lets through would become an out-of-bounds read on
the host (dictionary tables, FSST headers) or in HBM.  Seed images cover every
encoding: FFOR, DELTA, DICT (int and string), RLE, ALP, FSST, with zone maps.
CPU only (no GPU, no HIP)."""
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "duckdb-fastlane_amd" / "csrc"


@pytest.fixture(scope="module")
def fuzzer(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    out = tmp_path_factory.mktemp("fuzz") / "fuzz_reader"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", "-I", str(CSRC), str(ROOT / "tests" / "fuzz" / "fuzz_reader.cpp"),
                    "-o", str(out)], check=True)
    return out


def seed_images(fl, tmp_path):
    rng = np.random.default_rng(5)
    n = 5000
    imgs = {
        "lineitem_full": fl.gen_image("lineitem_full", 0.001),    # FFOR, DELTA, DICT strings, FSST
        "lineitem_dbl": fl.gen_image("lineitem_dbl", 0.001),      # ALP
        "mixed": fl.write_image([
            ("rle", fl.INT32, np.repeat(rng.integers(0, 9, n // 50), 50), fl.ENC_RLE),
            ("dict", fl.INT64, rng.integers(0, 5, n) * 1000003, fl.ENC_DICT),
            ("delta", fl.INT16, np.cumsum(rng.integers(0, 3, n)).astype(np.int16), fl.ENC_DELTA),
            ("alp", fl.DOUBLE, np.where(rng.random(n) < 0.1, rng.random(n), np.round(rng.normal(0, 99, n), 2)),
             fl.ENC_ALP),
            ("s", fl.VARCHAR, [("x" * int(k)) + "\xff" for k in rng.integers(0, 30, n)], fl.ENC_FSST),
        ], rowgroup=2048),
    }
    paths = []
    for name, img in imgs.items():
        p = tmp_path / f"{name}.fls"
        img.write(str(p))
        paths.append(p)
    return paths


def test_reader_survives_mutations_under_asan(fl, fuzzer, tmp_path):
    for i, p in enumerate(seed_images(fl, tmp_path)):
        r = subprocess.run([str(fuzzer), str(p), "1000", str(1000 + i)], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, f"{p.name}: sanitizer report\n{r.stderr[-4000:]}"
        assert r.stdout.startswith("iterations 1000"), r.stdout
