"""HBM-resident compressed images (DataChunk delivery).

The scan pipeline keeps a scanned file's compressed image in the GPU's HBM
(with the open-file cache entry): the first scan uploads each batch into it,
and later scans of the same unchanged file decode their row groups from it --
no staging copy, no H2D, only decoded bytes cross PCIe.  These tests check
that warm scans (resident image) deliver exactly what cold scans and scans
with the cache off (FLS_SCAN_RESIDENT_MB=0) deliver, filtered and unfiltered,
at 1 and 4 threads, and that the warm path is the one taken."""
import numpy as np
import pytest

from ext_harness import Ext

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ext(_built):
    e = Ext()
    yield e
    e.close()


@pytest.mark.parametrize("threads", [1, 4])
def test_warm_scans_match_cold_and_uncached(ext, fl, gpu, tmpfile, monkeypatch, capfd, threads):
    p = tmpfile(f"resident_{threads}.fls")
    fl.gen_image("lineitem_full", 0.05).write(p)
    monkeypatch.setenv("FLS_SCAN_RESIDENT_MB", "0")
    ref = ext.scan_count("read_fastlanes", p, threads=threads)[:2]
    ref_q6 = ext.scan_count("read_fastlanes", p, threads=threads, where=[(4, ">= 24"), (6, "<= 0.07")])[:2]
    monkeypatch.delenv("FLS_SCAN_RESIDENT_MB")
    monkeypatch.setenv("FLS_DEBUG", "1")
    capfd.readouterr()
    cold = ext.scan_count("read_fastlanes", p, threads=threads)[:2]
    warm = ext.scan_count("read_fastlanes", p, threads=threads)[:2]
    err = capfd.readouterr().err
    assert cold == ref and warm == ref
    assert "decoded from the HBM-resident image" in err
    warm_q6 = ext.scan_count("read_fastlanes", p, threads=threads, where=[(4, ">= 24"), (6, "<= 0.07")])[:2]
    assert warm_q6 == ref_q6


def test_rewritten_file_is_not_served_from_a_stale_image(ext, fl, gpu, tmpfile):
    """A file rewritten in place (new size / mtime: a new open-cache entry)
    is decoded from its own bytes, never from the old file's resident image."""
    import os
    import time
    p = tmpfile("rewritten.fls")
    fl.gen_image("lineitem", 0.02).write(p)
    a = ext.scan_count("read_fastlanes", p, threads=2)[:2]
    assert ext.scan_count("read_fastlanes", p, threads=2)[:2] == a      # warm
    time.sleep(0.01)
    fl.gen_image("lineitem", 0.03).write(p)
    os.utime(p)
    b = ext.scan_count("read_fastlanes", p, threads=2)[:2]
    assert b != a and b[0] == fl.gen_nrows("lineitem", 0.03)
    assert ext.scan_count("read_fastlanes", p, threads=2)[:2] == b
