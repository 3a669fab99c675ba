"""The HBM image budget (csrc/fls_resident.hpp).

The scan pipeline keeps scanned files' compressed bytes resident in HBM.
One byte budget per GPU covers every cached file; the least recently used
image no running scan holds is evicted first; fls_release_device_memory
frees every idle image.  The policy is host code, driven here on the CPU
through a small C++ driver (tests/resident_set_driver.cpp); the GPU tests in
test_resident_scan.py check the same behaviour through real scans."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    gxx = shutil.which("g++")
    if not gxx:
        pytest.skip("g++ not available")
    exe = tmp_path_factory.mktemp("resident") / "resident_set_driver"
    subprocess.run([gxx, "-std=c++17", "-O1", "-Wall", "-Werror", f"-I{ROOT / 'duckdb-fastlane_amd' / 'csrc'}",
                    str(ROOT / "tests" / "resident_set_driver.cpp"), "-o", str(exe)], check=True)

    def run(script: str):
        out = subprocess.run([str(exe)], input=script, capture_output=True, text=True, check=True).stdout
        return out.strip().splitlines()
    return run


def test_second_file_over_budget_evicts_the_older(driver):
    out = driver("""get 1 0 60 100
get 2 0 60 100
state 0
get 1 0 60 100
state 0""")
    assert out == ["new", "new evict1", "60 1 live 1", "new evict2", "60 1 live 1"]


def test_least_recently_used_goes_first(driver):
    out = driver("""get 1 0 30 100
get 2 0 30 100
get 3 0 30 100
get 1 0 30 100
get 4 0 30 100
state 0""")
    # file 1 was used again after 2 and 3, so 2 is the oldest
    assert out == ["new", "new", "new", "hit", "new evict2", "90 3 live 3"]


def test_an_image_a_scan_holds_is_never_evicted(driver):
    out = driver("""get 1 0 60 100
hold 1 0
get 2 0 60 100
state 0
drop 1 0
get 2 0 60 100
state 0""")
    assert out == ["new", "held", "none", "60 1 live 1", "ok", "new evict1", "60 1 live 1"]


def test_budget_is_per_gpu(driver):
    out = driver("""get 1 0 60 100
get 1 1 60 100
get 2 1 30 100
state 0
state 1
state -1""")
    assert out == ["new", "new", "new", "60 1 live 3", "90 2 live 3", "150 3 live 3"]


def test_image_larger_than_budget_is_not_made(driver):
    out = driver("""get 1 0 101 100
get 1 0 100 100
state 0""")
    assert out == ["none", "new", "100 1 live 1"]


def test_release_frees_idle_images_only(driver):
    out = driver("""get 1 0 10 100
get 2 0 20 100
get 3 1 40 100
hold 2 0
release 0
state 0
drop 2 0
release -1
state -1""")
    assert out == ["new", "new", "new", "held", "10", "20 1 live 2", "ok", "60", "0 0 live 0"]


def test_closed_file_drops_its_images_even_while_held(driver):
    out = driver("""get 1 0 10 100
get 1 1 10 100
hold 1 1
close 1
state -1
drop 1 1
state -1""")
    # the held image leaves the registry at once and is freed when the scan lets go
    assert out == ["new", "new", "held", "2", "0 0 live 1", "ok", "0 0 live 0"]


def test_evict_lru_skips_held_images(driver):
    out = driver("""get 1 0 10 100
get 2 0 10 100
hold 1 0
lru 0
lru 0
state 0""")
    assert out == ["new", "new", "held", "2", "-1", "10 1 live 1"]


def test_shards_of_one_file_share_a_gpu(driver):
    """a connection listing one GPU several times (the
    8-way split rehearsed on one GPU) keeps one image per shard there."""
    script = "\n".join(f"shard 1 0 {100 * g} {100 * (g + 1)} 10000" for g in range(8)) + "\nstate 0"
    out = driver(script)
    assert out == ["new replaced 0"] * 8 + ["800 8 live 8"]
    # the same shards again: all hits
    again = driver(script + "\n" + "\n".join(f"shard 1 0 {100 * g} {100 * (g + 1)} 10000" for g in range(8)))
    assert again[9:] == ["hit"] * 8


def test_other_split_replaces_idle_overlapping_shards_only(driver):
    out = driver("""shard 1 0 0 100 10000
shard 1 0 100 200 10000
shard 1 0 200 300 10000
hold 1 0
shard 1 0 0 300 10000
drop 1 0
shard 1 0 0 300 10000
state 0""")
    # a held shard (the first: hold takes any image of the file) overlapping
    # the new range is used as it is; once released, the whole-file request
    # replaces all three idle shards with one image
    assert out == ["new replaced 0", "new replaced 0", "new replaced 0", "held", "held", "ok",
                   "new replaced 3", "300 1 live 1"]
