"""The C-ABI shared libraries load and export every entry point their headers
declare (no GPU needed; no compute calls)."""
import ctypes as C
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADERS = {
    "flsgpu.h": "libflsgpu.so",
    "flswriter.h": "libflsgpu.so",
    "flscheck.h": "libflscheck.so",
}


def declared(header: Path):
    text = header.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//.*", "", text)
    return sorted(set(re.findall(r"\b(fls_[a-z0-9_]+)\s*\(", text)))


@pytest.mark.parametrize("hdr,lib", sorted(HEADERS.items()))
def test_exports(_built, hdr, lib):
    names = declared(ROOT / "include" / hdr)
    assert len(names) >= 2
    so = C.CDLL(str(ROOT / "duckdb-fastlane_amd" / lib))
    missing = [n for n in names if not hasattr(so, n)]
    assert not missing, f"{lib} lacks {missing}"


def test_extension_entry_points(_built):
    so = C.CDLL(str(ROOT / "duckdb-fastlane_amd" / "libfastlane_ext.so"))
    # DuckDB loads an extension through these two symbols (src/fastlane_extension.cpp:113-124)
    assert hasattr(so, "fastlane_init") and hasattr(so, "fastlane_version")
    so.fastlane_version.restype = C.c_char_p
    assert so.fastlane_version() == b"v1.3.2"


def test_no_gpu_needed_for_schema(fl, tmpfile):
    img = fl.gen_image("lineitem", 0.01)
    conn = fl.Connection()
    t = conn.read_image(img)
    assert t.ncols == 15 and t.nrows == 60175 and t.nrowgroups == 1
    s = t.schema()
    assert s[0][:2] == ("l_orderkey", fl.INT64) and s[4][1:4] == (fl.DECIMAL, 15, 2)
    assert [c[4] for c in s] == [8, 4, 4, 4, 8, 8, 8, 8, 16, 16, 4, 4, 4, 16, 16]


def test_open_errors(fl, tmpfile):
    conn = fl.Connection()
    with pytest.raises(fl.FlsError, match="Failed to open FastLanes file: nonexistent.fls"):
        conn.read_fls("nonexistent.fls")
    p = tmpfile("junk.fls")
    Path(p).write_bytes(b"not a fastlanes file at all" * 10)
    with pytest.raises(fl.FlsError) as e:
        conn.read_fls(p)
    assert e.value.code == -2
    # truncated image of a valid file
    img = fl.gen_image("c1", nrows=5000).tobytes()
    with pytest.raises(fl.FlsError):
        conn.read_image(img[:-40])
    # a chunk offset pointing past the footer is rejected up front
    import struct
    raw = bytearray(img)
    foff = struct.unpack_from("<Q", raw, len(raw) - 16)[0]
    ncols = struct.unpack_from("<I", raw, foff + 4)[0]
    p0 = foff + 32
    for _ in range(ncols):
        p0 += 6 + struct.unpack_from("<H", raw, p0 + 4)[0]
    struct.pack_into("<Q", raw, p0 + 4, foff + 1024)
    with pytest.raises(fl.FlsError, match="chunk out of bounds"):
        conn.read_image(bytes(raw))
