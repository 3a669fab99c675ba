#!/usr/bin/env python3
"""bench.py -- decoded values/s + achieved HBM GB/s of the MI355X FastLanes scan.

Metric (BASELINE.json): "decoded values/sec + achieved HBM GB/s, TPC-H SF100
lineitem scan at 1/2/4/8 GPU".  A step is ONE decode launch over every
resident vector of every column of this rank's row-group shard (compressed
input resident in HBM, decoded columns written to HBM): decode_kernel, or,
with l_comment's FSST chunks in the table, ONE fused_kernel that decodes the
main columns and the FSST strings side by side (round 5; FLS_FUSED=0: the
decode and FSST kernels of earlier rounds).  The default workload is the full
16-column lineitem (l_comment FSST-compressed).
Row groups are sharded contiguously over ranks with no data-path collective
(SURVEY.md 8(e)); torch.distributed over gloo (CPU tensors) only brackets the
timing (barrier, MAX of times, SUM of values) and gathers the per-rank
verification -- the scan has no exchange step, so no RCCL communicator is
created.  Rank r runs on GPU (local_rank mod visible GPUs): on a node with
fewer GPUs than ranks several ranks share one GPU, and config.ranks_per_gpu
says so (such a line rehearses the split; it is not a scaling point).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload lineitem_full]
                    [--scale 100] [--cpu-seconds 10] [--e2e-scale 10]

--gpus N without a torch.distributed launcher starts N ranks itself (one
process per GPU, before this process touches a GPU); under torchrun the
launcher's RANK / LOCAL_RANK / WORLD_SIZE are used.  Every rank checks every
decoded value of its shard on its GPU against the seeded generator
(libflscheck.so) after the timed region.  Rank 0 of a 1-GPU run also times
the CPU baseline (a FastLanes-shaped CPU decoder, oracle/flsfast.cpp, on the
host's cores) and the end-to-end rates into pinned host memory / DuckDB
DataChunks, which are never `value`.
"""
from __future__ import annotations

import argparse
import json
import statistics
import math
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s)
HBM_ACHIEVABLE_GBS = 6290.0  # measured achievable per GPU (MI355X_MICROARCH.md; SURVEY.md 8(d) "also vs 6.29")
PCIE_GBS = 63.0         # PCIe Gen5 x16 per GPU, spec (MI355X_MICROARCH.md)
WORKLOADS = ["lineitem_full", "lineitem", "lineitem_dbl", "c1", "c3", "c4"]


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", default="lineitem_full", choices=WORKLOADS)
    p.add_argument("--scale", type=float, default=100.0, help="lineitem scale factor")
    p.add_argument("--rows", type=int, default=0, help="row override (c1/c3/c4; 0 = config default)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    p.add_argument("--e2e-scale", type=float, default=10.0,
                   help="scale of the end-to-end (pinned host / DataChunk) measurement (0 = skip)")
    p.add_argument("--threads", type=int, default=0, help="host threads for encode / CPU baseline (0 = host cores)")
    p.add_argument("--no-verify", action="store_true", help="skip the full-shard GPU check")
    p.add_argument("--no-traffic", action="store_true",
                   help="skip the rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE child passes")
    p.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--e2e-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--dry-run", action="store_true",
                   help="launcher rehearsal on CPU: ranks, shards and the cross-rank reduction over gloo; "
                        "no GPU, no decode (tests/test_bench_launcher.py)")
    p.add_argument("--dry-run-node-gpus", type=int, default=0, help=argparse.SUPPRESS)
    return p.parse_args(argv)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def shard_range(nrg: int, rank: int, world: int):
    """Contiguous row-group range of `rank`: concatenating the
    ranks' ranges in rank order reproduces the table order; no collective."""
    return nrg * rank // world, nrg * (rank + 1) // world


# ---- host CPU facts ---------------------------------------------------------
def cgroup_cpu_quota() -> float | None:
    """CPUs the cgroup may use (cpu.max quota / period), None if unlimited."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                return int(q) / int(per)
        except (OSError, ValueError):
            pass
    try:  # cgroup v1
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return q / per
    except (OSError, ValueError):
        pass
    return None


def host_cores() -> dict:
    """The CPUs this process may run on: its affinity mask, capped by the
    cgroup CPU quota (the GPU box gives each GPU a quota of host cores)."""
    aff = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    usable = aff if quota is None else max(1, min(aff, math.floor(quota + 1e-9)))
    return {"usable": usable, "affinity": aff, "cgroup_quota": quota, "model": cpu_model()}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads(args, world_local: int = 1) -> int:
    if args.threads:
        return args.threads
    return max(1, host_cores()["usable"] // max(1, world_local))


# ---- launcher ---------------------------------------------------------------
def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_envs(n: int, port: int, base_env: dict) -> list[dict]:
    """Environment of each of n ranks started by this script (one per GPU)."""
    envs = []
    for r in range(n):
        e = dict(base_env)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                  "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        envs.append(e)
    return envs


def launch(args, argv) -> int:
    """--gpus N with no launcher: start N fresh ranks of this script before any
    GPU call here, wait for all of them, exit with the worst status.  Rank 0
    prints the JSON line."""
    envs = rank_envs(args.gpus, free_port(), os.environ)
    procs = [subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + list(argv), env=e) for e in envs]
    return wait_ranks(procs)


def wait_ranks(procs, poll_s: float = 0.2, grace_s: float = 30.0) -> int:
    """Wait for every rank; when one fails, stop the others (they would wait
    for it at the next barrier forever): SIGTERM, then SIGKILL after grace_s.
    Returns 0 or the failing rank's status."""
    first_bad = None
    while True:
        rcs = [p.poll() for p in procs]
        if first_bad is None:
            first_bad = next((rc for rc in rcs if rc not in (None, 0)), None)
            if first_bad is not None:
                log(f"launcher: a rank exited with status {first_bad}; stopping the others")
                for p in procs:
                    if p.poll() is None:
                        p.terminate()
                deadline = time.monotonic() + grace_s
        if all(rc is not None for rc in rcs):
            return first_bad if first_bad is not None else 0
        if first_bad is not None and time.monotonic() > deadline:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        time.sleep(poll_s)


# ---- measurement pieces -----------------------------------------------------
def e2e_child(args):
    cmd = [sys.executable, str(ROOT / "bench.py"), "--e2e-child", "--no-traffic", "--workload", args.workload,
           "--e2e-scale", str(args.e2e_scale), "--threads", str(args.threads)]
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
        if p.returncode != 0:
            return {"error": f"e2e child exited {p.returncode}: {p.stderr[-500:]}"}
        return json.loads(p.stdout.strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001 - the e2e numbers are reported beside the metric
        return {"error": repr(e)}


def measure_traffic(args):
    """HBM bytes per decode launch from rocprofv3 PMC counters, each counter in
    its own pass (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950).
    Runs as child processes BEFORE this process touches the GPU.  Corrections
    per MI355X_MICROARCH.md (HBM/rocprofv3): counters are in KiB; FETCH_SIZE
    reports half the bytes of 16 B/lane streaming reads -> x2."""
    import csv
    import shutil
    import tempfile
    if shutil.which("rocprofv3") is None:
        return None, "rocprofv3 not found"
    vals = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix=f"fls_pmc_{ctr.lower()}_", dir=os.environ.get("TMPDIR", "/tmp"))
        cmd = ["rocprofv3", "--pmc", ctr, "-d", d, "-o", "pmc", "--output-format", "csv", "--",
               sys.executable, str(ROOT / "bench.py"), "--pmc-child", "--steps", "2", "--warmup", "1",
               "--workload", args.workload, "--scale", str(args.scale), "--rows", str(args.rows),
               "--cpu-seconds", "0", "--e2e-scale", "0", "--no-verify", "--no-traffic"]
        # the child's upload rates no output placements: its rating launches
        # would be counted as decode dispatches (bytes per launch do not
        # depend on the placement)
        env = {**os.environ, "FLS_PLACEMENT_DECODE": "0", "FLS_PLACEMENT_TRIES": "1"}
        try:
            subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=600, env=env)
        except Exception as e:  # noqa: BLE001 - report, never fail the bench on profiling
            return None, f"rocprofv3 {ctr} pass failed: {e}"
        per = {}  # kernel -> samples (a step is the fused kernel, or decode_kernel plus the FSST kernels)
        for path in Path(d).rglob("*counter_collection.csv"):
            for r in csv.DictReader(open(path)):
                k = r.get("Kernel_Name", "")
                kind = ("fsst_sp" if "fsst_sp_kernel" in k else "fsst_cp" if "fsst_kernel" in k
                        else "fused" if "fused_kernel" in k else "decode" if "decode_kernel" in k else None)
                if kind and r.get("Counter_Name") == ctr:
                    per.setdefault(kind, []).append(float(r["Counter_Value"]))
        shutil.rmtree(d, ignore_errors=True)
        if "decode" not in per and "fused" not in per:
            return None, f"no {ctr} samples"
        # per step: every dispatch of the step's kernels (a table decode with
        # FSST columns runs several grids of each kind), over the child's
        # warmup + steps decode calls
        vals[ctr] = sum(sum(v) for v in per.values()) / 3.0 * 1024.0  # KiB -> bytes, per step
    return 2.0 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"], \
        f"rocprofv3 --pmc per launch: FETCH_SIZE x2 {2 * vals['FETCH_SIZE'] / 1e9:.3f} GB + " \
        f"WRITE_SIZE {vals['WRITE_SIZE'] / 1e9:.3f} GB"


def kernel_name(args) -> str:
    """the kernel(s) one step launches (launch_all in flsgpu.hip)"""
    if args.workload != "lineitem_full":
        return "fls::decode_kernel"
    if os.environ.get("FLS_FUSED", "") == "0":
        return "fls::decode_kernel + fls::fsst_kernel"
    return "fls::fused_kernel (main decode + FSST)"


def cpu_baseline(fl, args, nthreads: int, nrows_total: int, cores: dict):
    """FastLanes-shaped CPU decoder (oracle/flsfast.cpp: width-specialised
    lane loops, FFOR / DELTA / DICT / RLE / ALP fused per vector, FSST's
    classic decoder) on a bounded sample of the same workload, all usable host
    cores, output buffers the size of the sample (several GB, well beyond the
    host's L3) reused across passes, as the GPU reuses its HBM columns."""
    from oracle import flsfast, flsref
    nrg_total = (nrows_total + 65535) // 65536
    sample_rg = min(nrg_total, 512)
    img = fl.gen_image(args.workload, args.scale, args.rows, 0, sample_rg, nthreads)
    rf = flsref.RefFile(img)
    obs = [rf.out_width(c) for c in range(rf.ncols)]
    res = {}
    for build in flsfast.available():
        d = flsfast.Decoder(img, img.ptr, img.len, obs, rf.nrows, 0, rf.nrowgroups, build)
        d.decode(nthreads)  # first touch of the output pages
        t0 = time.perf_counter()
        n = d.decode(nthreads)
        one = time.perf_counter() - t0
        reps = max(1, int(args.cpu_seconds / 3 / max(one, 1e-6)))
        t0 = time.perf_counter()
        for _ in range(reps):
            n = d.decode(nthreads)
        dt = time.perf_counter() - t0
        t0 = time.perf_counter()
        reps1 = 0
        while reps1 == 0 or time.perf_counter() - t0 < args.cpu_seconds / 6:
            d.decode(1)
            reps1 += 1
        dt1 = time.perf_counter() - t0
        res[build] = {"value": n * reps / dt, "value_1core": n * reps1 / dt1, "passes": reps, "seconds": dt}
        del d
    best = max(res, key=lambda b: res[b]["value"])
    out_gb = rf.nrows * sum(obs) / 1e9
    return {
        "value": res[best]["value"],
        "unit": "values/s",
        "cores": nthreads,
        "kind": "port",
        "build": best,
        "value_1core": res[best]["value_1core"],
        "builds": res,
        "host": cores,
        "sample": f"{args.workload} row groups [0,{sample_rg}) = {rf.nrows} rows x {rf.ncols} cols "
                  f"({out_gb:.1f} GB decoded per pass, beyond L3), oracle/flsfast.cpp FastLanes-shaped decoder, "
                  f"{nthreads} threads ({cores['usable']} usable CPUs: affinity {cores['affinity']}, "
                  f"cgroup quota {cores['cgroup_quota']}), best of builds {list(res)}",
    }


def e2e_rates(fl, args, nthreads: int):
    """PCIe-inclusive rates (never `value`): the engine scan (compressed batch
    H2D -> decode -> D2H into pinned host memory, fls_scan_*) and read_fastlanes
    delivering zero-copy DataChunks through the executor harness (count-only
    sink), on an SF(--e2e-scale) file of the same workload."""
    import ctypes as C
    import tempfile
    wl = args.workload if args.workload.startswith("lineitem") else "lineitem"
    img = fl.gen_image(wl, args.e2e_scale, 0, 0, None, nthreads)
    t = fl.Connection([0]).read_image(img)
    ob = sum(t.column(c).out_bytes for c in range(t.ncols))
    for _ in t.scan():  # warm: pins the image, allocates the slots
        break
    passes = []
    for _ in range(3):
        rows = 0
        out = fl.RowGroup()
        t0 = time.perf_counter()
        fl._check(fl.lib.fls_scan_begin(t.h, None, 0, t.nrowgroups))
        while fl._check(fl.lib.fls_scan_next(t.h, C.byref(out))) == 1:
            rows += out.nrows
        passes.append((time.perf_counter() - t0, rows))
    dt, rows = min(passes)
    res = {"file": f"{wl} SF{args.e2e_scale:g}: {t.nrows} rows x {t.ncols} cols",
           "engine_scan_rows_s": rows / dt,
           "engine_scan_gbs": rows * ob / dt / 1e9,
           "engine_scan_frac_pcie": rows * ob / dt / 1e9 / PCIE_GBS,
           "engine_scan_note": "decoded column bytes delivered into pinned host memory (string_t 16 B; "
                               "FSST heap bytes not counted), best of 3 passes"}
    t.close()
    sys.path.insert(0, str(ROOT / "tests"))
    from ext_harness import Ext
    fd, path = tempfile.mkstemp(suffix=".fls", dir=os.environ.get("TMPDIR", "/tmp"))
    os.close(fd)
    try:
        img.write(path)
        e = Ext()
        # the first query of the file is cold (its compressed image crosses
        # PCIe and stays resident in HBM); the ones after it are warm
        n, sec = e.scan_rows("read_fastlanes", path, threads=nthreads)
        res[f"datachunk_cold_rows_s_{nthreads}t"] = n / sec
        for th in sorted({1, nthreads}):
            # warm queries vary run to run (4.0-6.9e8 rows/s at 16 threads on
            # one box in round 4): the median is the rate, the best and every
            # query's rate are reported beside it
            rates = []
            for _ in range(3 if th == 1 else 6):
                n, sec = e.scan_rows("read_fastlanes", path, threads=th)
                rates.append(n / sec)
            res[f"datachunk_rows_s_{th}t"] = statistics.median(rates)
            res[f"datachunk_best_rows_s_{th}t"] = max(rates)
            res[f"datachunk_all_rows_s_{th}t"] = [round(r) for r in rates]
        e.close()
    finally:
        os.unlink(path)
    res["datachunk_note"] = ("read_fastlanes -> DuckDB DataChunks (vectors reference the pinned row groups), "
                             "count-only sink, includes bind/open; datachunk_rows_s_*: MEDIAN of 3 (1 thread) / "
                             "6 (N threads) warm queries, datachunk_best_rows_s_*: their best, datachunk_all_rows_s_*: "
                             "each of them (warm: the file's compressed image resident in HBM from an earlier query, "
                             "FLS_SCAN_RESIDENT_MB); datachunk_cold_rows_s_*: the file's first query in a fresh "
                             "process connection (pinned buffers, streams and the HBM image made on the way)")
    return res


def verify_full(fl, t, args) -> tuple[int, int]:
    """Every decoded value of the resident shard vs the generator, on the GPU.
    Returns (mismatching values, values checked)."""
    mism = fl.check_device_table(t, args.workload, args.scale, args.rows)
    return int(sum(mism)), int(t.device_rows) * t.ncols


# ---- cross-rank reduction -----------------------------------------------------
# per-rank record: [seconds, values, achieved GB/s, kernel ms, algorithmic
# bytes per launch, mismatching values, values checked, row groups]
REC_FIELDS = ["seconds", "values", "achieved_gbs", "kernel_ms", "algo_bytes", "mismatches", "values_checked",
              "rowgroups"]


def gather_ranks(local: list[float], dist_on: bool) -> list[list[float]]:
    """All ranks' records, over gloo (CPU tensors): the bench needs no GPU
    collective, and gloo works whatever the rank -> GPU mapping is (RCCL
    refuses two ranks on one device)."""
    if not dist_on:
        return [list(local)]
    import torch
    import torch.distributed as dist
    x = torch.tensor(local, dtype=torch.float64)
    allx = [torch.zeros_like(x) for _ in range(dist.get_world_size())]
    dist.all_gather(allx, x)
    return [a.tolist() for a in allx]


def gather_objects(obj, dist_on: bool) -> list:
    if not dist_on:
        return [obj]
    import torch.distributed as dist
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def rank_device(local_rank: int, ngpus: int) -> int:
    """The GPU of a rank: its local rank, wrapped over the visible GPUs (a
    launcher that narrows visibility to one GPU per process gives ngpus=1)."""
    return local_rank % ngpus if ngpus > 0 else 0


def ranks_per_gpu(gpu_ids: list[str]) -> int:
    """Most ranks sharing one physical GPU (ids = host + device UUID)."""
    from collections import Counter
    return max(Counter(gpu_ids).values()) if gpu_ids else 1


def reduce_ranks(per_rank: list[list[float]]) -> dict:
    """Aggregate over ranks: the job's time is the slowest rank's, its values
    the sum (total values / max-over-GPUs wall time)."""
    return {"dt": max(r[0] for r in per_rank),
            "values": sum(r[1] for r in per_rank),
            "mean_achieved": sum(r[2] for r in per_rank) / len(per_rank),
            "hbm_gbs": sum(r[2] for r in per_rank),
            "mismatches": int(sum(r[5] for r in per_rank)),
            "checked": int(sum(r[6] for r in per_rank)),
            "rowgroups": [int(r[7]) for r in per_rank]}


def dry_run(args) -> None:
    """Launcher rehearsal (no GPU): every rank takes its shard of the
    workload's row groups, makes a synthetic per-rank record from it and the
    records go through the same gloo all_gather + reduction as a GPU run."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    import pkgload
    fl = pkgload.load()
    nrows = fl.gen_nrows(args.workload, args.scale, args.rows)
    nrg = (nrows + 65535) // 65536
    rg0, rg1 = shard_range(nrg, rank, world)
    rows = min(nrows, rg1 * 65536) - rg0 * 65536
    local = [1.0 + 0.25 * rank, float(rows), 100.0 * (rank + 1), 1.0, 0.0, 0.0, float(rows), float(rg1 - rg0)]
    per_rank = gather_ranks(local, world > 1)
    # the rank -> GPU mapping of a node with args.gpus visible devices, as a GPU run makes it
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    ids = gather_objects(f"host:gpu{rank_device(local_rank, args.dry_run_node_gpus or world)}", world > 1)
    # host threads each rank's encode would use: the node's usable cores split
    # over the ranks on the node, exactly as main() computes them
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    threads = gather_objects(host_threads(args, local_world if world > 1 else 1), world > 1)
    if rank == 0:
        red = reduce_ranks(per_rank)
        print(json.dumps({"dry_run": True, "n_gpus": world, "rowgroups": nrg, "rows": nrows,
                          "shards": [list(shard_range(nrg, r, world)) for r in range(world)],
                          "gpu_ids": ids, "ranks_per_gpu": ranks_per_gpu(ids), "host_threads": threads,
                          "usable_cores": host_cores()["usable"],
                          "reduced": red, "value": red["values"] / red["dt"]}), flush=True)
    if world > 1:
        dist.destroy_process_group()


# ---- main -------------------------------------------------------------------
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args, argv))
    if args.dry_run:
        dry_run(args)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))

    traffic, traffic_note = None, "not measured (multi-rank run or --no-traffic)"
    under_profiler = "rocprof" in os.environ.get("LD_PRELOAD", "") or any(k.startswith("ROCPROF") for k in os.environ)
    if under_profiler:
        traffic_note = "not measured (already running under rocprofv3)"
    if world == 1 and not args.no_traffic and not args.pmc_child and not under_profiler:
        traffic, traffic_note = measure_traffic(args)
        log(f"[traffic] {traffic_note}")
    if args.e2e_child:
        import pkgload
        print(json.dumps(e2e_rates(pkgload.load(), args, host_threads(args, 1))), flush=True)
        return
    # the PCIe-inclusive e2e block (never `value`) in its own process, before
    # this one touches the GPU: its scans' buffers land where a fresh process's
    # would, not among the HBM the metric's upload allocated and rated
    # 
    e2e = None
    if rank == 0 and world == 1 and args.e2e_scale > 0 and not args.pmc_child:
        e2e = e2e_child(args)

    import torch  # torch first: its HIP runtime is the one the engine binds to
    import torch.distributed as dist

    dist_on = world > 1
    if dist_on:
        dist.init_process_group("gloo")   # CPU bracket only: no data-path collective
    # this rank's GPU: its local rank wrapped over the visible GPUs
    dev = rank_device(local_rank, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    props = torch.cuda.get_device_properties(dev)
    gpu_id = f"{socket.gethostname()}:{getattr(props, 'uuid', '')}:{getattr(props, 'pci_bus_id', dev)}"
    gpu_ids = gather_objects(gpu_id, dist_on)
    rpg = ranks_per_gpu(gpu_ids)
    if rank == 0 and rpg > 1:
        log(f"[launcher] {world} ranks on {len(set(gpu_ids))} GPU(s): {rpg} ranks share a GPU "
            f"(a rehearsal of the {world}-way split, not a scaling point)")

    import pkgload
    fl = pkgload.load()
    cores = host_cores()
    nthreads = host_threads(args, local_world if dist_on else 1)

    nrows = fl.gen_nrows(args.workload, args.scale, args.rows)
    nrg = (nrows + 65535) // 65536
    rg0, rg1 = shard_range(nrg, rank, world)
    t_gen = time.perf_counter()
    img = fl.gen_image(args.workload, args.scale, args.rows, rg0, rg1, nthreads)
    t_gen = time.perf_counter() - t_gen
    log(f"[rank {rank}] encoded row groups [{rg0},{rg1}) of {nrg}: {img.len / 1e9:.2f} GB in {t_gen:.1f} s "
        f"({nthreads} threads)")

    conn = fl.Connection([dev])
    t = conn.read_image(img)
    t_up = time.perf_counter()
    t.device_upload()
    t_up = time.perf_counter() - t_up
    log(f"[rank {rank}] uploaded {img.len / 1e9:.2f} GB in {t_up:.2f} s; {t.device_rows} rows resident")

    for _ in range(args.warmup):
        t.device_decode()
    t.device_sync()

    def barrier():
        if dist_on:
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        t.device_decode()
    st = t.device_sync()
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0

    # roofline of this rank's decode launch (HIP events on the decode stream)
    avg_ms = st.kernel_ms_total / max(1, st.timed_launches)
    algo = st.algo_bytes
    achieved = algo / (avg_ms * 1e-3) / 1e9

    bad, checked = 0, 0
    if not args.no_verify:
        bad, checked = verify_full(fl, t, args)
        if bad:
            log(f"[rank {rank}] VERIFY FAILED: {bad} of {checked} values differ from the generator")

    local = [dt, float(st.values * args.steps), achieved, avg_ms, float(algo), float(bad), float(checked),
             float(rg1 - rg0)]
    per_rank = gather_ranks(local, dist_on)
    red = reduce_ranks(per_rank)
    dt, total_vals, bad_total, checked_total = red["dt"], red["values"], red["mismatches"], red["checked"]
    mean_achieved = red["mean_achieved"]

    ncols_main = t.ncols
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(fl, args, nthreads, nrows, cores)

    if rank == 0:
        big = args.workload.startswith("lineitem")
        cfg = {"workload": args.workload + (f" SF{args.scale:g}" if big else ""),
               "rows": nrows, "columns": ncols_main, "rowgroups": nrg,
               "rowgroups_per_gpu": red["rowgroups"], "parallelism": f"rowgroup-shard x{world}",
               "ranks_per_gpu": rpg, "physical_gpus": len(set(gpu_ids)),
               "step": "one decode launch over all resident vectors of the shard (HBM -> HBM)",
               "compressed_bytes_rank0": img.len, "decoded_bytes_rank0": int(st.out_bytes),
               "verified_values_bit_exact": checked_total if (bad_total == 0 and checked_total > 0) else 0,
               "verified_mismatches": bad_total,
               "verification": "every decoded value of every rank's shard vs the seeded generator, on the GPU "
                               "(libflscheck.so)" if not args.no_verify else "skipped (--no-verify)"}
        line = {
            "metric": f"decoded values/sec ({args.workload}" + (f" SF{args.scale:g} full scan)" if big else ")"),
            "value": total_vals / dt,
            "unit": "values/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",  # fixed SF100 total, row groups split over ranks
            "vs_baseline": None,
            "dtype": "u8..u64 integer unpack -> int32/int64/string_t" + (" + f64 (ALP)" if "dbl" in args.workload
                                                                          else ""),
            "data": {"lineitem_full": "synthetic (seeded TPC-H-like generator, all 16 columns, l_comment FSST)",
                     "lineitem": "synthetic (seeded TPC-H-like generator, l_comment excluded)",
                     "lineitem_dbl": "synthetic (seeded TPC-H-like generator, DECIMAL columns as DOUBLE/ALP)"}.get(
                args.workload, "synthetic (seeded generator)"),
            "config": cfg,
            "hbm_gbs": red["hbm_gbs"],
            "roofline": {"bound": "hbm", "achieved": mean_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": mean_achieved / HBM_PEAK_GBS,
                         "achievable": HBM_ACHIEVABLE_GBS, "frac_achievable": mean_achieved / HBM_ACHIEVABLE_GBS,
                         "traffic": traffic / 1e9 if traffic else None,
                         "traffic_unit": "GB per launch (HBM, PMC)", "traffic_note": traffic_note,
                         "kernel": kernel_name(args),
                         "kernel_ms": avg_ms,
                         "algo_bytes_per_launch": algo,
                         "algo_bytes_split": {"packed": int(st.packed_bytes), "meta": int(st.meta_bytes),
                                              "out": int(st.out_bytes)},
                         "per_rank": [{"achieved_gbs": r[2], "kernel_ms": r[3], "algo_bytes": r[4]}
                                      for r in per_rank] if world > 1 else None},
            "per_rank": [dict({"rank": i, "gpu": gpu_ids[i]}, **{k: (int(v) if k in ("values", "mismatches",
                                                                                    "values_checked", "rowgroups")
                                                                    else v) for k, v in zip(REC_FIELDS, r)})
                         for i, r in enumerate(per_rank)] if world > 1 else None,
            "e2e": e2e,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.destroy_process_group()
    if bad_total:
        sys.exit(3)


if __name__ == "__main__":
    main()
