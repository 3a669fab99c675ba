"""fls_read_fls keeps recently opened files mapped with their validated
metadata (MappedFile cache keyed by device, inode, size and mtime): an
unchanged file reopens without revalidation, a rewritten one is validated
again.  CPU only (opening a file touches no GPU)."""
import os
import time

import numpy as np
import pytest


def _open(fl, path):
    conn = fl.Connection([0])
    return conn, conn.read_fls(str(path))


def test_reopen_unchanged_file_same_table(fl, tmp_path):
    p = tmp_path / "a.fls"
    fl.gen_image("lineitem", 0.01).write(str(p))
    c1, t1 = _open(fl, p)
    c2, t2 = _open(fl, p)
    assert (t1.ncols, t1.nrows, t1.nrowgroups) == (t2.ncols, t2.nrows, t2.nrowgroups)
    assert t1.schema() == t2.schema()
    t1.close()
    # the second table keeps the shared mapping alive after the first closes
    assert t2.rowgroup_rows(0) == t2.nrows
    t2.close()


def test_rewritten_file_is_reread_and_revalidated(fl, tmp_path):
    p = tmp_path / "b.fls"
    fl.gen_image("lineitem", 0.01).write(str(p))
    _, t = _open(fl, p)
    assert t.ncols == 15
    t.close()
    rng = np.random.default_rng(3)
    fl.write_image([("x", fl.INT32, rng.integers(0, 9, 5000), fl.ENC_AUTO)]).write(str(p))
    _, t = _open(fl, p)
    assert (t.ncols, t.nrows) == (1, 5000)
    t.close()
    # same size, different bytes, later mtime: validated again, and rejected
    good = p.read_bytes()
    bad = bytearray(good)
    bad[300:340] = b"\xff" * 40  # inside the first chunk's header / metadata
    time.sleep(0.01)
    p.write_bytes(bytes(bad))
    st = os.stat(p)
    os.utime(p, ns=(st.st_atime_ns, st.st_mtime_ns + 1_000_000))
    with pytest.raises(Exception):
        _open(fl, p)


def test_release_memory_hook_registered(_built):
    """fastlane_release_memory(): the SQL hook that hands idle pinned memory back."""
    import sys
    sys.path.insert(0, str(__import__("pathlib").Path(__file__).parent))
    from ext_harness import Ext
    e = Ext()
    try:
        assert e.scalar0("fastlane_release_memory") == "0"
    finally:
        e.close()


@pytest.mark.gpu
def test_idle_pinned_memory_capped_and_trimmed(fl, gpu, monkeypatch):
    """A scan's pipeline goes back to the connection when its table closes;
    the pinned host batches it keeps are capped by bytes per GPU
    (FLS_IDLE_PINNED_MB) and fls_connection_trim frees them on demand."""
    import numpy as np
    img = fl.gen_image("lineitem", 0.2)   # 19 row groups: several 8-row-group batches
    conn = fl.Connection([0])
    monkeypatch.setenv("FLS_IDLE_PINNED_MB", "4096")
    t = conn.read_image(img)
    nrg = t.nrowgroups
    rows = sum(1 for _ in t.scan())
    t.close()
    big = conn.trim(1 << 62)              # nothing freed, report what is idle
    assert rows == nrg and big > 64 << 20
    monkeypatch.setenv("FLS_IDLE_PINNED_MB", "64")
    t = conn.read_image(img)
    sum(1 for _ in t.scan())
    t.close()
    assert conn.trim(1 << 62) <= 64 << 20   # capped when the scan handed its pipeline back
    assert conn.trim(0) == 0                # and all of it released on demand
    t = conn.read_image(img)                # a later scan builds a new pipeline
    assert sum(1 for _ in t.scan()) == nrg
    t.close()
    conn.close()
