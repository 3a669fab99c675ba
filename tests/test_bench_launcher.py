"""bench.py's multi-GPU entry point, rehearsed on CPU:
`bench.py --gpus N` without a torch.distributed launcher starts N ranks
itself; each rank takes its contiguous row-group shard and the per-rank
records go through the same gloo all_gather + reduction a GPU run uses (the
bench creates no RCCL communicator): job time = slowest rank, values = sum
over ranks.  test_bench_two_ranks_one_gpu runs the real thing on the GPU."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

import bench

ROOT = Path(__file__).resolve().parents[1]


def test_rank_envs_one_process_per_gpu():
    envs = bench.rank_envs(4, 29511, {"PATH": "/bin"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert all(e["WORLD_SIZE"] == "4" and e["LOCAL_WORLD_SIZE"] == "4" for e in envs)
    assert all(e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29511" and e["PATH"] == "/bin"
               for e in envs)


def test_reduce_ranks_max_time_sum_values():
    recs = [[2.0, 100.0, 5000.0, 1.0, 0, 0, 100.0, 3], [2.5, 120.0, 4000.0, 1.1, 0, 2, 120.0, 4]]
    r = bench.reduce_ranks(recs)
    assert r["dt"] == 2.5 and r["values"] == 220.0 and r["mismatches"] == 2 and r["checked"] == 220
    assert r["mean_achieved"] == 4500.0 and r["hbm_gbs"] == 9000.0 and r["rowgroups"] == [3, 4]


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_ranks_and_reduces(_built, n):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--dry-run",
                        "--workload", "lineitem", "--scale", "100"],
                       capture_output=True, text=True, env=env, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout          # only rank 0 prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["rowgroups"] == 9156 and out["rows"] == 600037902
    shards = out["shards"]
    assert shards[0][0] == 0 and shards[-1][1] == 9156
    assert all(a[1] == b[0] for a, b in zip(shards, shards[1:]))          # contiguous, in rank order
    assert max(b - a for a, b in shards) - min(b - a for a, b in shards) <= 1
    red = out["reduced"]
    assert red["values"] == 600037902 and red["checked"] == 600037902
    assert red["dt"] == 1.0 + 0.25 * (n - 1)                               # the slowest rank's time
    assert red["rowgroups"] == [b - a for a, b in shards]
    assert out["value"] == pytest.approx(600037902 / red["dt"])
    assert out["ranks_per_gpu"] == 1 and len(set(out["gpu_ids"])) == n   # one GPU per rank on an n-GPU node


def test_gpus_8_node_rehearsal(_built):
    """the driver's 8-GPU run must not be the first time
    this configuration executes.  Eight ranks over gloo on the CPU, as on an
    8-GPU node (--dry-run-node-gpus 8): SF100's 9,156 row groups split
    1,144 / 1,145, contiguous and in rank order; one GPU per rank; each rank's
    encode threads are the node's usable cores divided by 8; only rank 0
    prints, and the reduction takes the slowest rank's time and every rank's
    values."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "8", "--dry-run", "--dry-run-node-gpus",
                        "8", "--workload", "lineitem_full", "--scale", "100"],
                       capture_output=True, text=True, env=env, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout          # only rank 0 prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["rowgroups"] == 9156 and out["rows"] == 600037902
    sizes = [b - a for a, b in out["shards"]]
    assert sorted(set(sizes)) == [1144, 1145] and sum(sizes) == 9156
    assert sizes.count(1145) == 9156 - 8 * 1144
    assert out["shards"][0][0] == 0 and out["shards"][-1][1] == 9156
    assert all(a[1] == b[0] for a, b in zip(out["shards"], out["shards"][1:]))
    assert out["gpu_ids"] == [f"host:gpu{r}" for r in range(8)] and out["ranks_per_gpu"] == 1
    assert out["host_threads"] == [max(1, out["usable_cores"] // 8)] * 8
    red = out["reduced"]
    assert red["values"] == 600037902 and red["rowgroups"] == sizes and red["dt"] == 1.0 + 0.25 * 7


def test_rank_device_wraps_over_visible_gpus():
    assert [bench.rank_device(r, 8) for r in range(8)] == list(range(8))
    assert [bench.rank_device(r, 1) for r in range(4)] == [0, 0, 0, 0]     # narrowed / 1-GPU lease
    assert [bench.rank_device(r, 2) for r in range(4)] == [0, 1, 0, 1]
    assert bench.ranks_per_gpu(["a", "b", "a", "a"]) == 3 and bench.ranks_per_gpu(["a", "b"]) == 1


def test_two_ranks_share_one_gpu_dry_run(_built):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--dry-run", "--dry-run-node-gpus",
                        "1", "--workload", "lineitem", "--scale", "1"],
                       capture_output=True, text=True, env=env, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["ranks_per_gpu"] == 2 and out["gpu_ids"] == ["host:gpu0", "host:gpu0"]


@pytest.mark.gpu
def test_bench_two_ranks_one_gpu(_built):
    """bench.py --gpus 2 end to end on the GPU (both ranks on GPU 0 of a 1-GPU
    lease): each rank decodes and verifies its contiguous shard; the line
    carries both ranks' records and every value of the table is verified."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    r = subprocess.run([sys.executable, "-u", str(ROOT / "bench.py"), "--gpus", "2", "--scale", "1",
                        "--steps", "3", "--warmup", "1", "--cpu-seconds", "0", "--e2e-scale", "0", "--no-traffic"],
                       capture_output=True, text=True, env=env, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    cfg = out["config"]
    assert out["n_gpus"] == 2 and cfg["rows"] == 6001215 and cfg["columns"] == 16
    assert cfg["rowgroups_per_gpu"] == [46, 46] and cfg["parallelism"] == "rowgroup-shard x2"
    assert cfg["ranks_per_gpu"] * cfg["physical_gpus"] >= 2
    pr = out["per_rank"]
    assert [p["rank"] for p in pr] == [0, 1] and [p["rowgroups"] for p in pr] == [46, 46]
    assert all(p["mismatches"] == 0 for p in pr)
    assert sum(p["values_checked"] for p in pr) == 6001215 * 16
    assert cfg["verified_values_bit_exact"] == 6001215 * 16 and cfg["verified_mismatches"] == 0
    assert out["value"] > 0 and sum(p["values"] for p in pr) == 6001215 * 16 * 3


def test_wait_ranks_stops_the_others_when_one_fails():
    # rank 1 fails at once; rank 0 would otherwise wait at a barrier for ever
    import time
    hang = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(600)"])
    fail = subprocess.Popen([sys.executable, "-c", "import sys; sys.exit(3)"])
    t0 = time.monotonic()
    try:
        assert bench.wait_ranks([hang, fail], poll_s=0.05, grace_s=5) == 3
    finally:
        if hang.poll() is None:
            hang.kill()
    assert hang.poll() is not None and time.monotonic() - t0 < 30


def test_wait_ranks_all_ok():
    procs = [subprocess.Popen([sys.executable, "-c", "pass"]) for _ in range(3)]
    assert bench.wait_ranks(procs, poll_s=0.05) == 0
