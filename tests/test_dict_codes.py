"""Dictionary-coded delivery (fls_scan_dict_codes).

A delivered DICT VARCHAR / BLOB column crosses PCIe as 1- or 2-byte codes
plus the row group's string_t dictionary instead of 16-byte string_t records,
and read_fastlanes hands DuckDB dictionary vectors (the reference's string
columns: /root/reference/src/fastlanes_facade.cpp:157-172).  The GPU produces
the codes with the DICT decode path gathering from an identity table, so the
codes are the chunk's stored codes; these tests check them against the
generator's strings and the string_t delivery, filtered and unfiltered."""
import numpy as np
import pytest

from ext_harness import Ext

pytestmark = pytest.mark.gpu

DICT_COLS = (8, 9, 13, 14)      # l_returnflag, l_linestatus, l_shipinstruct, l_shipmode


@pytest.fixture(scope="module")
def ext(_built):
    e = Ext()
    yield e
    e.close()


def _strings(arr, dct):
    """codes + dictionary (string_t records, host) -> python bytes"""
    import ctypes as C
    rec = dct.reshape(-1, 16)
    out = []
    for code in arr.tolist():
        r = rec[code]
        n = int(r[:4].view(np.uint32)[0])
        if n <= 12:
            out.append(bytes(r[4:4 + n]))
        else:
            out.append(C.string_at(int(r[8:16].view(np.uint64)[0]), n))
    return out


@pytest.mark.parametrize("rowgroup_filter", [None, [(0, ">", 3000)]])
def test_scan_delivers_dict_codes(fl, gpu, rowgroup_filter):
    wl, sf = "lineitem", 0.02
    img = fl.gen_image(wl, sf)
    t = fl.Connection([0]).read_image(img)
    n = t.nrows
    t.set_filter(rowgroup_filter or [])
    t.dict_codes(True)
    got = {c: [] for c in DICT_COLS}
    rows = []
    widths = set()
    for first, arrays, dicts in t.scan_dicts():
        for c in DICT_COLS:
            assert dicts[c] is not None, c
            widths.add(arrays[c].dtype.itemsize)
            got[c] += _strings(arrays[c], dicts[c])
        rows.append(len(arrays[0]) // 8)
    assert widths == {1}
    okey = fl.gen_values(wl, 0, 0, n, np.int64, sf)
    keep = okey > 3000 if rowgroup_filter else np.ones(n, bool)
    assert sum(rows) == int(keep.sum())
    for c in DICT_COLS:
        exp = fl.gen_strings(wl, c, 0, n, sf)
        assert got[c] == [e for e, k in zip(exp, keep) if k], c
    # a filter on a dictionary column keeps it in string_t form (the filter reads it)
    t.set_filter([(14, "=", "AIR")])
    for first, arrays, dicts in t.scan_dicts():
        assert dicts[14] is None and dicts[13] is not None
    t.dict_codes(False)
    t.set_filter([])
    for first, arrays, dicts in t.scan_dicts():
        assert all(d is None for d in dicts)
        break


@pytest.mark.parametrize("threads", [1, 4])
def test_read_fastlanes_dictionary_vectors_match_flat(ext, fl, gpu, tmpfile, monkeypatch, threads):
    """read_fastlanes with dictionary vectors (default) and with string_t
    delivery (FLS_READ_DICT=0, in a child process: the knob is read once)
    produce the same checksum; every string matches the generator."""
    import subprocess
    import sys
    p = tmpfile("li.fls")
    fl.gen_image("lineitem", 0.02).write(p)
    rows, h, _ = ext.scan_count("read_fastlanes", p, threads=threads)
    code = ("import sys; sys.path.insert(0, 'tests'); from ext_harness import Ext; e = Ext(); "
            f"r, h, _ = e.scan_count('read_fastlanes', {p!r}, threads={threads}); print(r, h)")
    out = subprocess.run([sys.executable, "-c", code], env={**__import__('os').environ, "FLS_READ_DICT": "0"},
                         capture_output=True, text=True, timeout=300, cwd=str(__import__('pathlib').Path(__file__).parents[1]))
    assert out.returncode == 0, out.stderr
    assert out.stdout.split() == [str(rows), str(h)]
    names, types, got = ext.query("read_fastlanes", p, proj=[14, 13, 0], threads=threads)
    n = len(got)
    okey = fl.gen_values("lineitem", 0, 0, n, np.int64, 0.02).tolist()
    ship = [x.decode() for x in fl.gen_strings("lineitem", 14, 0, n, 0.02)]
    instr = [x.decode() for x in fl.gen_strings("lineitem", 13, 0, n, 0.02)]
    assert sorted((int(r[2]), r[0], r[1]) for r in got) == sorted(zip(okey, ship, instr))
