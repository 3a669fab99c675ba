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


def _resident(fl, dev=0):
    return fl.Connection.resident_info(dev)


def test_two_files_over_budget_evict_the_older(ext, fl, gpu, tmpfile, monkeypatch):
    """One HBM budget per GPU over every cached file: with
    room for one image, scanning a second file evicts the first one's (the
    least recently used image no scan holds), and the first file then scans
    bit-exactly again from its bytes on disk."""
    a, b = tmpfile("budget_a.fls"), tmpfile("budget_b.fls")
    fl.gen_image("lineitem_full", 0.1).write(a)
    fl.gen_image("lineitem_full", 0.11).write(b)
    import os
    big = max(os.path.getsize(a), os.path.getsize(b))
    monkeypatch.setenv("FLS_SCAN_RESIDENT_MB", "0")
    ref_a = ext.scan_count("read_fastlanes", a, threads=4)[:2]
    ref_b = ext.scan_count("read_fastlanes", b, threads=4)[:2]
    fl.Connection.release_device_memory()
    assert _resident(fl) == (0, 0)
    # room for the larger file, not for both
    monkeypatch.setenv("FLS_SCAN_RESIDENT_MB", str(big // (1 << 20) + 2))
    assert ext.scan_count("read_fastlanes", a, threads=4)[:2] == ref_a
    bytes_a, n = _resident(fl)
    assert n == 1 and bytes_a >= os.path.getsize(a) // 2
    assert ext.scan_count("read_fastlanes", b, threads=4)[:2] == ref_b
    bytes_b, n = _resident(fl)
    assert n == 1 and bytes_b != bytes_a          # a's image made room for b's
    assert ext.scan_count("read_fastlanes", a, threads=4)[:2] == ref_a   # after eviction: from disk again
    assert _resident(fl) == (bytes_a, 1)
    assert ext.scan_count("read_fastlanes", a, threads=4)[:2] == ref_a   # warm, from its image
    # a budget with room for both keeps both
    monkeypatch.setenv("FLS_SCAN_RESIDENT_MB", str(2 * (big // (1 << 20)) + 4))
    assert ext.scan_count("read_fastlanes", b, threads=4)[:2] == ref_b
    assert _resident(fl) == (bytes_a + bytes_b, 2)
    fl.Connection.release_device_memory()


def _hbm_free():
    """Free HBM of the current device from the HIP runtime the engine loaded
    (hipMemGetInfo; not torch, whose own bundled runtime may not come up next
    to it in a process that already holds the device)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")
    free, tot = ctypes.c_size_t(), ctypes.c_size_t()
    assert hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(tot)) == 0
    return free.value


def test_release_returns_the_hbm(ext, fl, gpu, tmpfile):
    """fastlane_release_memory() frees the resident images as well as the idle
    pinned host memory: the device's free memory (hipMemGetInfo) grows by
    the images' bytes, and the next scan is still exact."""
    p = tmpfile("release.fls")
    fl.gen_image("lineitem_full", 0.2).write(p)
    fl.Connection.release_device_memory()
    first = ext.scan_count("read_fastlanes", p, threads=4)[:2]
    held, n = _resident(fl)
    assert n == 1 and held > 0
    free_before = _hbm_free()
    assert ext.scalar0("fastlane_release_memory") == "0"
    assert _resident(fl) == (0, 0)
    free_after = _hbm_free()
    assert free_after - free_before >= held - (4 << 20), (free_before, free_after, held)
    assert ext.scan_count("read_fastlanes", p, threads=4)[:2] == first


def test_image_holds_only_this_gpus_shard(ext, fl, gpu, tmpfile, monkeypatch):
    """A GPU's image holds its shard of the table: with the table
    split over two devices (GPU 0 listed twice), GPU 0 holds one image per
    shard (round 6: the registry keys images by shard, so the split rehearsed
    on one GPU keeps both), together about the file, and both decode
    exactly; a later unsplit scan replaces the two idle shards with one
    image."""
    import os
    p = tmpfile("shard.fls")
    fl.gen_image("lineitem", 0.2).write(p)
    fl.Connection.release_device_memory()
    monkeypatch.setenv("FLS_SCAN_RESIDENT_MB", "0")
    ref = ext.scan_count("read_fastlanes", p, threads=4)[:2]
    monkeypatch.delenv("FLS_SCAN_RESIDENT_MB")
    con = fl.Connection([0, 0])
    t = con.read_fls(p)
    sch = t.schema()
    rows = sum(len(cols[0]) // sch[0][4] for _, cols in t.scan(cols=[0]))
    assert rows == ref[0]
    held, n = _resident(fl)
    size = os.path.getsize(p)
    assert n == 2 and 0.9 * size < held < 1.05 * size   # two half-size shard images on GPU 0
    t.close()
    t1 = fl.Connection([0]).read_fls(p)
    rows1 = sum(len(cols[0]) // sch[0][4] for _, cols in t1.scan(cols=[0]))
    assert rows1 == ref[0]
    held1, n1 = _resident(fl)
    assert n1 == 1 and 0.9 * size < held1 < 1.05 * size   # one whole-file image replaced the shards
    t1.close()
    fl.Connection.release_device_memory()
