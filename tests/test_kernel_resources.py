"""Register budgets of the shipped gfx950 kernels, read from the built
library's code-object metadata on the CPU (scripts/kernel_resources.py).
They pin the occupancy design points DESIGN.md states: the encoder kernels
spill nothing (a 6-wave build that spilled 6 VGPRs wrote wrong T=32 DELTA
rows), the main decode kernel fits 4 waves per SIMD,
the default code-parallel FSST kernel 6, the segmented FSST kernel 5 (its LDS
admits about that many) with no spill."""
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "scripts"))
LIB = ROOT / "duckdb-fastlane_amd" / "libflsgpu.so"


@pytest.fixture(scope="module")
def res():
    if not LIB.exists():
        pytest.skip("libflsgpu.so not built")
    import kernel_resources
    r = kernel_resources.resources(str(LIB))
    assert r, "no gfx950 code object in libflsgpu.so"
    return r


def _find(res, *parts):
    hits = {k: v for k, v in res.items() if all(p in k for p in parts)}
    assert hits, parts
    return hits


def test_encoder_kernels_do_not_spill(res):
    for name, r in {**_find(res, "encode_kernel"), **_find(res, "encode_rle_kernel")}.items():
        assert r["vgpr_spill"] == 0 and r["scratch"] == 0, (name, r)
    narrow = _find(res, "encode_kernelIj")  # T <= 32: 5 waves per SIMD
    assert all(r["vgpr"] <= 80 for r in narrow.values()), narrow  # 6 waves per SIMD fit (scalar wave index)


def test_decode_kernel_fits_four_waves(res):
    for name, r in _find(res, "decode_kernel").items():
        assert r["vgpr"] + r["agpr"] <= 128, (name, r)


def test_default_fsst_kernel_fits_six_waves(res):
    # fsst_kernel<Kind::Cp, SMALL, QUEUE>: the code-parallel kernel (chunks without segment tables)
    hits = _find(res, "fsst_kernelILNS0_4KindE1E")
    assert len(hits) == 4, hits
    assert all(r["vgpr"] <= 80 and r["vgpr_spill"] == 0 for r in hits.values()), hits


def test_segmented_fsst_kernel_fits_five_waves_without_spill(res):
    # fsst_kernel<Kind::Seg, SMALL, QUEUE>: the segmented kernel (every chunk the writer produces)
    hits = _find(res, "fsst_kernelILNS0_4KindE0E")
    assert len(hits) == 4, hits
    for name, r in hits.items():
        assert r["vgpr"] <= 96 and r["vgpr_spill"] == 0 and r["scratch"] == 0, (name, r)


def test_product_library_holds_only_the_default_fsst_kernels(res):
    """the wrong-output cost ablations and the losing
    variants live in the experiment library (csrc/fls_fsst_lab.hip, make lab)
    only.  The product library's FSST kernels are exactly the segmented and
    code-parallel kernels (small / any strings x range / piece queue) plus the
    string-parallel policy kernel and the writer's compressor."""
    fsst = sorted(k for k in res if "fsst" in k)
    decoders = [k for k in fsst if "fsst_kernel" in k]
    assert len(decoders) == 8, decoders
    assert all("4KindE" in k for k in decoders), decoders   # no variant / ring-cap template arguments
    others = [k for k in fsst if "fsst_kernel" not in k]
    assert sorted(o.split("fsst_")[1].split("_kernel")[0] for o in others) == ["compress", "sp"], others
