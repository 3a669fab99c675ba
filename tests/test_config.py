"""Deployment knobs: the defaults the public headers and INTEGRATION.md state
are the library's (include/flsgpu.h said 512 for
FLS_IDLE_PINNED_MB while the code used 1024).  CPU only: no compute calls.

The library keeps every knob's default in one table (csrc/fls_config.hpp) and
reads the knobs only through it; fls_config_default / fls_config_value /
fls_config_count / fls_config_name report it.
"""
import ctypes as C
import os
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def fl():
    import pkgload
    return pkgload.load()


def _doc_table():
    """INTEGRATION.md's knob table: name -> default."""
    rows = re.findall(r"^\| `(FLS_[A-Z_]+)` \| ([0-9]+) \|", (ROOT / "INTEGRATION.md").read_text(), re.M)
    assert rows, "INTEGRATION.md lost its knob table"
    return {k: int(v) for k, v in rows}


def _header_defaults():
    """Defaults stated in include/*.h comments: 'FLS_X, default N' / 'FLS_X (default N'."""
    out = {}
    for h in sorted((ROOT / "include").glob("*.h")):
        text = re.sub(r"\s*\n\s*\*?\s*", " ", h.read_text())  # join comment lines
        for name, num in re.findall(r"(FLS_[A-Z_]+)[,(]? ?\(?default ([0-9][0-9,]*)", text):
            out.setdefault(name, []).append((h.name, int(num.replace(",", ""))))
    return out


def test_library_table_matches_integration_table(fl):
    lib = fl.config()
    doc = _doc_table()
    assert set(lib) == set(doc), f"knobs only in the library: {set(lib) - set(doc)}; only in INTEGRATION.md: {set(doc) - set(lib)}"
    for k, (d, _) in lib.items():
        assert d == doc[k], f"{k}: library default {d}, INTEGRATION.md says {doc[k]}"


def test_header_defaults_match_library(fl):
    lib = fl.config()
    found = _header_defaults()
    # the headers document at least these three
    for k in ("FLS_IDLE_PINNED_MB", "FLS_SCAN_RESIDENT_MB", "FLS_SCAN_HOST_BATCHES", "FLS_SCAN_STRLEN"):
        assert k in found, f"{k}: no 'default N' in include/*.h"
    for k, where in found.items():
        assert k in lib, f"{k} documented with a default in {where[0][0]} but not a library knob"
        for h, v in where:
            assert v == lib[k][0], f"{h}: {k} default {v}, library {lib[k][0]}"


def test_value_follows_environment(fl, monkeypatch):
    monkeypatch.setenv("FLS_COPY_BATCH", "3")
    assert fl.config()["FLS_COPY_BATCH"] == (8, 3)
    monkeypatch.delenv("FLS_COPY_BATCH")
    assert fl.config()["FLS_COPY_BATCH"] == (8, 8)


def test_unknown_knob_is_an_argument_error(fl):
    v = C.c_int64()
    assert fl.lib.fls_config_default(b"FLS_NO_SUCH_KNOB", C.byref(v)) == -3
    assert fl.lib.fls_config_value(None, C.byref(v)) == -3
    assert fl.lib.fls_config_name(fl.lib.fls_config_count()) is None


def test_every_knob_read_goes_through_the_table():
    """No deployment knob is read with getenv() outside fls_config.hpp (a
    second default would drift from the table again)."""
    import pkgload  # noqa: F401
    names = set(_doc_table())
    srcs = list((ROOT / "duckdb-fastlane_amd" / "csrc").glob("*.[ch]*")) + \
        list((ROOT / "duckdb-fastlane_amd" / "extension" / "src").rglob("*.[ch]pp"))
    bad = []
    for f in srcs:
        if f.name == "fls_config.hpp":
            continue
        for m in re.finditer(r'getenv\("(FLS_[A-Z_]+)"\)', f.read_text(errors="replace")):
            if m.group(1) in names:
                bad.append(f"{f.name}: {m.group(1)}")
    assert not bad, bad
