#!/usr/bin/env python3
"""bench.py -- decoded values/s + achieved HBM GB/s of the MI355X FastLanes scan.

Metric (BASELINE.json): "decoded values/sec + achieved HBM GB/s, TPC-H SF100
lineitem scan at 1/2/4/8 GPU".  A step is ONE fused decode launch over every
resident vector of every column of this rank's row-group shard (compressed
input resident in HBM, decoded columns written to HBM).  Row groups are sharded
contiguously over ranks with no data-path collective; the
torch.distributed barrier / MAX reduction only brackets the timing.

N=1 workload = the metric's own configuration (SF100 fits one GPU: ~11 GB
compressed + ~77 GB decoded).  Inputs are synthetic (seeded TPC-H-like
generator, fls_gen.hpp) and encoded by this repo's CPU writer before timing.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload lineitem]
                    [--scale 100] [--cpu-seconds 10]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", default="lineitem",
                   choices=["lineitem", "c1", "c3", "c4", "lineitem_full", "lineitem_dbl"])
    p.add_argument("--scale", type=float, default=100.0, help="lineitem scale factor")
    p.add_argument("--rows", type=int, default=0, help="row override (c1/c3/c4; 0 = config default)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    p.add_argument("--threads", type=int, default=0, help="host threads for encode / CPU baseline")
    p.add_argument("--verify-rowgroups", type=int, default=3)
    p.add_argument("--no-traffic", action="store_true",
                   help="skip the rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE child passes")
    p.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    return p.parse_args()


def shard_range(nrg: int, rank: int, world: int):
    """Contiguous row-group range of `rank`: concatenating the
    ranks' ranges in rank order reproduces the table order; no collective."""
    return nrg * rank // world, nrg * (rank + 1) // world


def measure_traffic(args):
    """HBM bytes per decode launch from rocprofv3 PMC counters, each counter in
    its own pass (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950).
    Runs as child processes BEFORE this process touches the GPU.  Corrections
    per MI355X_MICROARCH.md (HBM/rocprofv3): counters are in KiB; FETCH_SIZE
    reports half the bytes of 16 B/lane streaming reads -> x2."""
    import csv
    import shutil
    import subprocess
    import tempfile
    if shutil.which("rocprofv3") is None:
        return None, "rocprofv3 not found"
    vals = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix=f"fls_pmc_{ctr.lower()}_", dir=os.environ.get("TMPDIR", "/tmp"))
        cmd = ["rocprofv3", "--pmc", ctr, "-d", d, "-o", "pmc", "--output-format", "csv", "--",
               sys.executable, str(ROOT / "bench.py"), "--pmc-child", "--steps", "2", "--warmup", "1",
               "--workload", args.workload, "--scale", str(args.scale), "--rows", str(args.rows),
               "--cpu-seconds", "0", "--verify-rowgroups", "0", "--no-traffic"]
        try:
            subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=600)
        except Exception as e:  # noqa: BLE001 - report, never fail the bench on profiling
            return None, f"rocprofv3 {ctr} pass failed: {e}"
        per = {}  # kernel -> samples (a step is decode_kernel, plus the FSST kernels for FSST columns)
        for path in Path(d).rglob("*counter_collection.csv"):
            for r in csv.DictReader(open(path)):
                k = r.get("Kernel_Name", "")
                kind = ("fsst_sp" if "fsst_sp_kernel" in k else "fsst_cp" if "fsst_kernel" in k
                        else "decode" if "decode_kernel" in k else None)
                if kind and r.get("Counter_Name") == ctr:
                    per.setdefault(kind, []).append(float(r["Counter_Value"]))
        shutil.rmtree(d, ignore_errors=True)
        if "decode" not in per:
            return None, f"no {ctr} samples"
        # per step: every dispatch of the step's kernels (a table decode with
        # FSST columns runs several grids of each kind), over the child's
        # warmup + steps decode calls
        vals[ctr] = sum(sum(v) for v in per.values()) / 3.0 * 1024.0  # KiB -> bytes, per step
    return 2.0 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"], \
        f"rocprofv3 --pmc per launch: FETCH_SIZE x2 {2 * vals['FETCH_SIZE'] / 1e9:.3f} GB + " \
        f"WRITE_SIZE {vals['WRITE_SIZE'] / 1e9:.3f} GB"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_threads(args) -> int:
    if args.threads:
        return args.threads
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        return max(1, int(env))
    return max(1, min(16, os.cpu_count() or 1))


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(fl, args, nthreads: int, nrows_total: int):
    """Oracle (CPU restatement, 'port') on a bounded sample of the same workload."""
    from oracle import flsref
    nrg_total = (nrows_total + 65535) // 65536
    sample_rg = min(nrg_total, 128)
    img = fl.gen_image(args.workload, args.scale, args.rows, 0, sample_rg, nthreads)
    rf = flsref.RefFile(img)
    vals_per_pass = rf.nrows * rf.ncols
    fsst = {c for c in range(rf.ncols) if rf.column(c)[1] == fl.VARCHAR and fl.gen_dict_string(args.workload, c, 0) is None}

    def one_pass(nth):
        for c in range(rf.ncols):
            if c in fsst:  # free text: the oracle's FSST decoder into offsets + bytes
                rf.decode_strings_column(c, nth)
            else:
                rf.decode_column(c, nth)

    # one pass to size the run, then repeat within the budget
    t0 = time.perf_counter()
    one_pass(nthreads)
    one = time.perf_counter() - t0
    reps = max(1, int(args.cpu_seconds / max(one, 1e-6)))
    t0 = time.perf_counter()
    for _ in range(reps):
        one_pass(nthreads)
    dt = time.perf_counter() - t0
    # the same restatement on one core (SURVEY.md 8(d) asks for both numbers)
    t0 = time.perf_counter()
    reps1 = 0
    while reps1 == 0 or time.perf_counter() - t0 < args.cpu_seconds / 4:
        one_pass(1)
        reps1 += 1
    dt1 = time.perf_counter() - t0
    return {
        "value": vals_per_pass * reps / dt,
        "value_1core": vals_per_pass * reps1 / dt1,
        "cpu_model": cpu_model(),
        "unit": "values/s",
        "cores": nthreads,
        "kind": "port",
        "sample": f"{args.workload} row groups [0,{sample_rg}) = {rf.nrows} rows x {rf.ncols} cols, "
                  f"oracle/flsref.c (gcc -O3), {nthreads} threads, {reps} passes in {dt:.1f} s; "
                  f"1 thread: {reps1} passes in {dt1:.1f} s",
    }


def verify(fl, t, args, rg_list):
    """Bit-exact check of sampled row groups against the generator ground truth."""
    first = t.row_offset
    sch = t.schema()
    for rg in rg_list:
        r0 = rg * 65536
        n = t.rowgroup_rows(rg)
        for c, (name, ty, _, _, ob) in enumerate(sch):
            got = t.device_copy_out(c, r0, n)
            if ty == fl.VARCHAR:
                dic = {}
                k = 0
                while True:
                    s = fl.gen_dict_string(args.workload, c, k)
                    if s is None:
                        break
                    dic[k] = s.encode()
                    k += 1
                if dic:
                    codes = fl.gen_values(args.workload, c, first + r0, n, np.uint32, args.scale, args.rows)
                    exp = [dic[int(x)] for x in codes]
                else:  # free text (l_comment, FSST)
                    exp = fl.gen_strings(args.workload, c, first + r0, n, args.scale, args.rows)
                if fl.string_t_decode(got) != exp:
                    return f"{name} rg {rg}"
            else:
                exp = fl.gen_values(args.workload, c, first + r0, n, fl.NP_DTYPE[ty], args.scale, args.rows)
                if not np.array_equal(got.view(fl.NP_DTYPE[ty]), exp):
                    return f"{name} rg {rg}"
    return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    traffic, traffic_note = None, "not measured (multi-rank run or --no-traffic)"
    under_profiler = "rocprof" in os.environ.get("LD_PRELOAD", "") or any(k.startswith("ROCPROF") for k in os.environ)
    if under_profiler:
        traffic_note = "not measured (already running under rocprofv3)"
    if world == 1 and not args.no_traffic and not args.pmc_child and not under_profiler:
        traffic, traffic_note = measure_traffic(args)
        log(f"[traffic] {traffic_note}")

    import torch  # torch first: its HIP runtime is the one the engine binds to
    import torch.distributed as dist

    dist_on = world > 1
    # this rank's GPU: its local rank, unless the launcher already narrowed the
    # visible devices to one per process
    dev = local_rank if torch.cuda.device_count() > local_rank else 0
    if dist_on:
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", device_id=torch.device("cuda", dev))

    import pkgload
    fl = pkgload.load()
    nthreads = host_threads(args)
    if dist_on:
        nthreads = max(1, nthreads // max(1, int(os.environ.get("LOCAL_WORLD_SIZE", world))))

    nrows = fl.gen_nrows(args.workload, args.scale, args.rows)
    nrg = (nrows + 65535) // 65536
    rg0, rg1 = shard_range(nrg, rank, world)
    t_gen = time.perf_counter()
    img = fl.gen_image(args.workload, args.scale, args.rows, rg0, rg1, nthreads)
    t_gen = time.perf_counter() - t_gen
    log(f"[rank {rank}] encoded row groups [{rg0},{rg1}) of {nrg}: {img.len / 1e9:.2f} GB in {t_gen:.1f} s")

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

    local_vals = st.values * args.steps
    if dist_on:
        x = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        dt = float(x.item())
        v = torch.tensor([local_vals], dtype=torch.float64, device="cuda")
        dist.all_reduce(v, op=dist.ReduceOp.SUM)
        total_vals = float(v.item())
    else:
        total_vals = float(local_vals)

    # roofline of the (single, fused) decode kernel on this rank
    avg_ms = st.kernel_ms_total / max(1, st.timed_launches)
    algo = st.algo_bytes
    achieved = algo / (avg_ms * 1e-3) / 1e9

    bad = None
    if args.verify_rowgroups > 0:
        n_local = rg1 - rg0
        picks = sorted({0, n_local // 2, n_local - 1})[: args.verify_rowgroups]
        bad = verify(fl, t, args, picks)
        if bad:
            log(f"[rank {rank}] VERIFY FAILED: {bad}")

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(fl, args, nthreads, nrows)

    if rank == 0:
        cfg = {"workload": f"{args.workload}" + (f" SF{args.scale:g}" if args.workload == "lineitem" else ""),
               "rows": nrows, "columns": t.ncols, "rowgroups": nrg,
               "rowgroups_per_gpu": rg1 - rg0, "parallelism": f"rowgroup-shard x{world}",
               "step": "one fused decode launch over all resident vectors (HBM -> HBM)",
               "compressed_bytes_per_gpu": img.len, "decoded_bytes_per_gpu": int(st.out_bytes),
               "verified_rowgroups_bit_exact": bad is None and args.verify_rowgroups > 0}
        line = {
            "metric": "decoded values/sec (TPC-H lineitem full scan)" if args.workload == "lineitem"
            else f"decoded values/sec ({args.workload})",
            "value": total_vals / dt,
            "unit": "values/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",  # fixed SF100 total, row groups split over ranks
            "vs_baseline": None,
            "dtype": "int64/int32/string_t (integer unpack)" if args.workload != "lineitem_dbl"
            else "int64/int32/string_t + f64 (ALP)",
            "data": {"lineitem": "synthetic (seeded TPC-H-like generator, l_comment excluded)",
                     "lineitem_full": "synthetic (seeded TPC-H-like generator, l_comment FSST text)",
                     "lineitem_dbl": "synthetic (seeded TPC-H-like generator, DECIMAL columns as DOUBLE/ALP)"}.get(
                args.workload, "synthetic (seeded generator)"),
            "config": cfg,
            "hbm_gbs": achieved * world,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic / 1e9 if traffic else None,
                         "traffic_unit": "GB per launch (HBM, PMC)", "traffic_note": traffic_note,
                         "kernel": "fls::decode_kernel" + (" + fls::fsst_kernel" if args.workload == "lineitem_full" else ""),
                         "kernel_ms": avg_ms,
                         "algo_bytes_per_launch": algo,
                         "algo_bytes_split": {"packed": int(st.packed_bytes), "meta": int(st.meta_bytes),
                                              "out": int(st.out_bytes)}},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.destroy_process_group()
    if bad:
        sys.exit(3)


if __name__ == "__main__":
    main()
