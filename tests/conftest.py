import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: full-size property tests (1e9 rows)")


def _make(d: Path):
    subprocess.run(["make", "-s", "-j3", "-C", str(d)], check=True)


@pytest.fixture(scope="session", autouse=True)
def _built():
    # idempotent in-tree builds (oracle C restatement, engine, DuckDB glue)
    _make(ROOT / "oracle")
    _make(ROOT / "duckdb-fastlane_amd")
    yield


@pytest.fixture(scope="session")
def fl(_built):
    import pkgload
    return pkgload.load()


@pytest.fixture(scope="session")
def ref(_built):
    from oracle import flsref
    return flsref


@pytest.fixture(scope="session")
def gpu(fl):
    n = fl.device_count()
    assert n > 0, "no HIP device visible: GPU tests must run on an MI355X"
    return n


@pytest.fixture
def tmpfile(tmp_path):
    return lambda name: str(tmp_path / name)


def nthreads():
    return min(16, os.cpu_count() or 1)
