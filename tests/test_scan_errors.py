"""Scan pipeline failure handling (flsgpu.hip scan_acquire /
scan_release): a batch refill that cannot be enqueued (an allocation failure,
injected here with FLS_TEST_FAIL_ENQUEUE) must turn into an error for every
consumer waiting for that batch and for every later acquire -- not a hang of
the DuckDB scan threads."""
import ctypes as C
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_failed_refill_errors_instead_of_hanging(fl, gpu, monkeypatch):
    monkeypatch.setenv("FLS_SCAN_BATCH", "1")     # one row group per batch: a refill per row group
    n = 6 * 65536
    img = fl.write_image([("v", fl.INT32, np.arange(n, dtype=np.int32), fl.ENC_FFOR)])
    t = fl.Connection([0]).read_image(img)
    assert t.nrowgroups == 6
    # scan_begin enqueues batches 1 and 2 (two slots); the third enqueue -- the
    # refill when row group 0 is handed out -- fails
    monkeypatch.setenv("FLS_TEST_FAIL_ENQUEUE", "3")
    fl._check(fl.lib.fls_scan_begin(t.h, None, 0, 6))
    results = {}

    def consumer(i):
        out = fl.RowGroup()
        rc = fl.lib.fls_scan_acquire(t.h, C.byref(out))
        results[i] = (rc, out.rowgroup if rc == 1 else None, fl.last_error() if rc < 0 else "")

    threads = [threading.Thread(target=consumer, args=(i,), daemon=True) for i in range(4)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=60)
    assert not any(th.is_alive() for th in threads), "a consumer hangs after the failed refill"
    delivered = sorted(r[1] for r in results.values() if r[0] == 1)
    errors = [r for r in results.values() if r[0] < 0]
    assert errors and all("injected batch enqueue failure" in r[2] for r in errors), results
    assert set(delivered) <= {0, 1}
    for rg in delivered:
        assert fl.lib.fls_scan_release(t.h, rg) == 0
    # the error is sticky for later acquires too
    out = fl.RowGroup()
    assert fl.lib.fls_scan_acquire(t.h, C.byref(out)) < 0
    # and a new scan starts clean
    monkeypatch.delenv("FLS_TEST_FAIL_ENQUEUE")
    got = np.concatenate([cols[0] for _, cols in t.scan()])
    assert np.array_equal(got.view(np.int32), np.arange(n, dtype=np.int32))
