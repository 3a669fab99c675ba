"""Without a GPU the product fails loudly:
the file opens and binds on any host (footer, schema), but every decode --
the engine scan, the device-resident upload and read_fastlanes -- reports
FLS_ERR_DEVICE instead of falling back to a CPU decode.  Runs only where no
HIP device is visible (this CPU container); skipped on the GPU box."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def nogpu_file(fl, tmp_path_factory):
    if fl.device_count() > 0:
        pytest.skip("a HIP device is visible: the no-GPU contract is checked on CPU-only hosts")
    p = tmp_path_factory.mktemp("nogpu") / "c1.fls"
    # BASELINE C1's shape: INT32, base 1,000,000 + U[0, 128) (W = 7 after FFOR)
    rng = np.random.default_rng(42)
    x = (1_000_000 + rng.integers(0, 128, 1_000_000)).astype(np.int32)
    fl.write_image([("data", fl.INT32, x, fl.ENC_FFOR)]).write(str(p))
    return str(p)


def test_open_and_schema_need_no_gpu(fl, nogpu_file):
    t = fl.Connection().read_fls(nogpu_file)
    assert t.nrows == 1_000_000 and t.nrowgroups == 16
    assert t.schema()[0][0] == "data"


def test_decode_fails_with_device_error(fl, nogpu_file):
    t = fl.Connection().read_fls(nogpu_file)
    with pytest.raises(fl.FlsError) as ei:
        list(t.scan())
    assert ei.value.code == -4 and "device" in str(ei.value).lower()
    with pytest.raises(fl.FlsError) as ei:
        t.device_upload()
    assert ei.value.code == -4


def test_read_fastlanes_binds_then_fails_loudly(nogpu_file):
    from ext_harness import Ext, ExtError
    e = Ext()
    try:
        with pytest.raises(ExtError, match="FastLanes scan failed"):
            e.scan_count("read_fastlanes", nogpu_file, threads=1)
    finally:
        e.close()
