"""C5 coverage: TPC-H SF100 lineitem (all 16 columns) checked value by value
on one GPU, and the in-process multi-GPU paths -- the device-resident table
split into per-GPU parts (fls_device_upload) and the sharded scan -- on every
visible GPU, or on GPU 0 listed twice when the box has one (same code path:
one part / pipeline per listed device, contiguous row-group ranges)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _devices(fl, want=2):
    n = fl.device_count()
    return list(range(n)) if n >= want else [0] * want


def test_device_resident_parts_bit_exact(fl, gpu):
    img = fl.gen_image("lineitem_full", 1.0)
    conn = fl.Connection([0, 0])
    t = conn.read_image(img)
    t.device_upload()
    parts = t.device_parts()
    assert len(parts) == 2 and [p.device for p in parts] == [0, 0]
    assert parts[0].rg_begin == 0 and parts[0].rg_end == parts[1].rg_begin and parts[1].rg_end == t.nrowgroups
    assert parts[0].first_row == 0 and parts[1].first_row == parts[0].nrows
    assert sum(p.nrows for p in parts) == t.nrows == t.device_rows
    for _ in range(2):
        t.device_decode()
    st = t.device_sync()
    assert st.timed_launches == 2 and st.values == 16 * t.nrows
    assert 0 < st.kernel_ms <= st.kernel_ms_total
    assert fl.check_device_table(t, "lineitem_full", 1.0) == [0] * 16
    # one-part accessors refuse a split table
    with pytest.raises(fl.FlsError, match="resident on 2 GPUs"):
        t.device_column(0)
    # copies spanning the part boundary equal the one-part table's
    one = fl.Connection([0]).read_image(img)
    one.device_upload()
    one.device_decode()
    one.device_sync()
    b = parts[1].first_row
    for c in (0, 4, 8, 10):  # l_orderkey, l_quantity, l_returnflag (inline string_t), l_shipdate
        assert np.array_equal(t.device_copy_out(c, b - 3000, 7000), one.device_copy_out(c, b - 3000, 7000))
    # the per-part check can fail: corrupt a value of the second part only
    p, _ = t.device_part_column(1, 0)
    hip = ctypes.CDLL("libamdhip64.so.7")
    bad = (ctypes.c_uint8 * 8)(*([0x5A] * 8))
    assert hip.hipMemcpy(ctypes.c_void_p(p + 8 * 777), bad, 8, 1) == 0
    assert fl.check_device_table(t, "lineitem_full", 1.0)[0] == 1


def test_every_visible_gpu_scan_and_resident(fl, ref, gpu, monkeypatch):
    """Every visible GPU (GPU 0 twice on a one-GPU box): the sharded scan
    delivers every row group in order, bit-exact vs the oracle, and the
    resident table splits into one part per GPU, checked on each GPU."""
    monkeypatch.setenv("FLS_SCAN_BATCH", "2")
    devs = _devices(fl)
    img = fl.gen_image("lineitem", 0.2)
    rf = ref.RefFile(img)
    conn = fl.Connection(devs)
    t = conn.read_image(img)
    got = list(t.scan(cols=[0, 3, 14]))
    assert [r // 65536 for r, _ in got] == list(range(rf.nrowgroups))
    for first, cols in got:
        rg = first // 65536
        for c in (0, 3):
            assert np.array_equal(cols[c], rf.decode(c, rg))
    t.device_upload()
    parts = t.device_parts()
    assert [p.device for p in parts] == devs[:len(parts)]
    assert len(parts) == min(len(devs), t.nrowgroups)
    t.device_decode()
    st = t.device_sync()
    assert st.values == 15 * t.nrows
    assert fl.check_device_table(t, "lineitem", 0.2) == [0] * 15


def test_lineitem_full_sf100_bit_exact(fl, gpu):
    """C5's table at full size on one GPU: 600,037,902 rows x 16 columns
    (l_comment FSST), every decoded value and heap byte vs the generator."""
    import os
    img = fl.gen_image("lineitem_full", 100.0, 0, 0, None, min(16, len(os.sched_getaffinity(0))))
    t = fl.Connection([0]).read_image(img)
    assert t.nrows == 600037902 and t.nrowgroups == 9156
    t.device_upload()
    t.device_decode()
    st = t.device_sync()
    assert st.values == 16 * t.nrows
    assert fl.check_device_table(t, "lineitem_full", 100.0) == [0] * 16


def test_eight_way_split_on_one_gpu(fl, gpu, tmp_path):
    """the 8-way engine split, rehearsed on one GPU
    (Connection([0] * 8): eight pipelines, eight resident parts, eight shard
    images, all on GPU 0).  lineitem_full SF1 has 92 row groups: shards of
    11 / 12, not multiples of the scan batch (8).  Checked: row-group order
    through scan(), every value of two columns vs the generator, the eight
    shard images, the device parts' boundaries, and every value of all 16
    columns of the device-resident decode.  A correctness rehearsal only:
    one physical GPU measures no scaling."""
    img = fl.gen_image("lineitem_full", 1.0)
    path = tmp_path / "l8.fls"
    img.write(str(path))
    fl.Connection.release_device_memory()
    t = fl.Connection([0] * 8).read_fls(str(path))
    N, n = t.nrowgroups, t.nrows
    assert N == 92 and n == 6001215
    names = [s[0] for s in t.schema()]
    ck, cd = names.index("l_orderkey"), names.index("l_shipdate")
    got = list(t.scan(cols=[ck, cd]))
    assert [first // 65536 for first, _ in got] == list(range(N))
    keys = np.concatenate([cols[ck].view(np.int64) for _, cols in got])
    days = np.concatenate([cols[cd].view(np.int32) for _, cols in got])
    assert np.array_equal(keys, fl.gen_values("lineitem_full", ck, 0, n, np.int64))
    assert np.array_equal(days, fl.gen_values("lineitem_full", cd, 0, n, np.int32))
    held, images = fl.Connection.resident_info(0)
    assert images == 8, (held, images)
    assert 0.9 * path.stat().st_size < held < 1.05 * path.stat().st_size
    t.device_upload()
    parts = t.device_parts()
    bounds = [N * g // 8 for g in range(9)]
    assert [(p.rg_begin, p.rg_end) for p in parts] == list(zip(bounds[:-1], bounds[1:]))
    assert sorted({p.rg_end - p.rg_begin for p in parts}) == [11, 12]
    assert [p.device for p in parts] == [0] * 8 and sum(p.nrows for p in parts) == n
    t.device_decode()
    st = t.device_sync()
    assert st.values == 16 * n
    assert fl.check_device_table(t, "lineitem_full", 1.0) == [0] * 16
    t.close()
    fl.Connection.release_device_memory()
