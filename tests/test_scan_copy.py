"""The scan's D2H by copy kernel (FLS_SCAN_COPY_KERNEL=1, the default: decoded
columns and string heaps into pinned host memory; csrc/fls_filter.hip
host_copy_kernel)
deliver byte for byte what the DMA engines (=0, hipMemcpyAsync) deliver:
ragged batches, resident and streamed images, full-width and narrowed
delivery, a filtered scan, every string by content."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _scan(fl, t, narrow, filt):
    t.set_filter(filt or [])
    t.narrow(narrow)
    sch = t.schema()
    out = None
    for first, arrays in t.scan():
        if out is None:
            out = [[] for _ in arrays]
        for c, a in enumerate(arrays):
            # string_t records point into the scan's pinned heaps: compared by
            # content, decoded while the row group is held
            out[c].append(fl.string_t_decode(a) if sch[c][1] in (fl.VARCHAR, fl.BLOB) else a)
    t.narrow(False)
    t.set_filter([])
    return out


def _same(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        if isinstance(x, list):
            assert x == y
        else:
            assert np.array_equal(x, y)


@pytest.mark.parametrize("resident", ["65536", "0"])
@pytest.mark.parametrize("narrow,filt", [(False, None), (True, None), (False, [(0, "<=", 300000)])])
def test_copy_kernel_matches_dma(fl, gpu, monkeypatch, resident, narrow, filt):
    monkeypatch.setenv("FLS_SCAN_BATCH", "3")  # 23 row groups: ragged last batch
    monkeypatch.setenv("FLS_SCAN_RESIDENT_MB", resident)
    t = fl.Connection([0]).read_image(fl.gen_image("lineitem_full", 0.25))
    got = {}
    for arm in ("1", "0", "1"):  # kernel, DMA, kernel again (a warm resident image)
        monkeypatch.setenv("FLS_SCAN_COPY_KERNEL", arm)
        got.setdefault(arm, []).append(_scan(fl, t, narrow, filt))
    ref = got["0"][0]
    assert sum(len(x) for x in ref[0]) > 0
    for k in got["1"]:
        assert len(k) == len(ref)
        for c in range(len(ref)):
            _same(k[c], ref[c])
    sch = t.schema()
    if not narrow and not filt:
        ok = [c for c in range(t.ncols) if sch[c][0] == "l_orderkey"][0]
        keys = np.concatenate(got["1"][0][ok]).view(np.int64)
        assert keys.size == t.nrows and keys[0] == 1 and np.all(np.diff(keys) >= 0)
        sc = [c for c in range(t.ncols) if sch[c][0] == "l_comment"][0]
        strs = [s for part in got["1"][0][sc] for s in part]
        assert strs[:3] == fl.gen_strings("lineitem_full", sc, 0, 3, scale=0.25)
