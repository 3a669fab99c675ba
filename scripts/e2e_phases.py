#!/usr/bin/env python3
"""Where the end-to-end (file -> pinned host / DataChunk) time goes: open
(mmap + footer), first fls_scan_begin (string_t tables, image pinning, slot
buffers), the scan loop; cold (new table) and warm (same table again); then
read_fastlanes DataChunks through the executor harness at 1 and N threads,
twice each.
    python scripts/e2e_phases.py [--workload lineitem_full] [--scale 10] [--threads 16]"""
import argparse
import ctypes as C
import os
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def scan_pass(fl, t):
    out = fl.RowGroup()
    rows = 0
    t0 = time.perf_counter()
    fl._check(fl.lib.fls_scan_begin(t.h, None, 0, t.nrowgroups))
    t1 = time.perf_counter()
    while fl._check(fl.lib.fls_scan_next(t.h, C.byref(out))) == 1:
        rows += out.nrows
    t2 = time.perf_counter()
    return rows, t1 - t0, t2 - t1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="lineitem_full")
    ap.add_argument("--scale", type=float, default=10)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--arms", default="", help="interleaved env arms for the N-thread DataChunk scan: "
                                               "'name:VAR=v,VAR2=v;name2:...' (same file, same box)")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import pkgload
    fl = pkgload.load()
    img = fl.gen_image(a.workload, a.scale, 0, 0, None, a.threads)
    fd, path = tempfile.mkstemp(suffix=".fls", dir=os.environ.get("TMPDIR", "/tmp"))
    os.close(fd)
    img.write(path)
    gb = img.len / 1e9
    img.close()
    print(f"{a.workload} SF{a.scale:g}: {gb:.2f} GB file", flush=True)
    try:
        conn = fl.Connection([0])
        for tag in ("cold", "warm-table"):
            t0 = time.perf_counter()
            t = conn.read_fls(path)
            t_open = time.perf_counter() - t0
            for p in range(2):
                rows, t_begin, t_loop = scan_pass(fl, t)
                print(f"{tag} pass {p}: open {t_open * 1e3:.1f} ms, scan_begin {t_begin * 1e3:.1f} ms, "
                      f"loop {t_loop * 1e3:.1f} ms -> {rows / t_loop / 1e6:.1f} M rows/s loop, "
                      f"{rows / (t_open + t_begin + t_loop) / 1e6:.1f} M rows/s incl. open+begin", flush=True)
                t_open = 0.0
            t.close()
        conn.close()
        from ext_harness import Ext
        e = Ext()
        for th in sorted({1, a.threads}):
            for rep in range(2):
                n, sec = e.scan_rows("read_fastlanes", path, threads=th)
                print(f"DataChunks {th} threads rep {rep}: {n} rows in {sec * 1e3:.1f} ms = {n / sec / 1e6:.1f} M rows/s",
                      flush=True)
        if a.arms:
            import statistics
            arms = []
            for spec in a.arms.split(";"):
                name, _, kv = spec.partition(":")
                arms.append((name, dict(x.split("=", 1) for x in kv.split(",") if x)))
            res = {name: [] for name, _ in arms}
            for _ in range(a.reps):
                for name, env in arms:
                    saved = {k: os.environ.get(k) for k in env}
                    os.environ.update(env)
                    try:
                        n, sec = e.scan_rows("read_fastlanes", path, threads=a.threads)
                    finally:
                        for k, v in saved.items():
                            if v is None:
                                os.environ.pop(k, None)
                            else:
                                os.environ[k] = v
                    res[name].append(n / sec)
            for name, v in res.items():
                print(f"arm {name}: DataChunks {a.threads} threads median {statistics.median(v) / 1e6:.1f} M rows/s "
                      f"(best {max(v) / 1e6:.1f}, worst {min(v) / 1e6:.1f}) over {len(v)}: "
                  + " ".join(f"{x / 1e6:.1f}" for x in v), flush=True)
        # the phase profile of the N-thread scan (read_fastlanes.cpp ReadProfile, printed on stderr)
        os.environ["FLS_READ_PROFILE"] = "1"
        sys.stderr.flush()
        n, sec = e.scan_rows("read_fastlanes", path, threads=a.threads)
        print(f"DataChunks {a.threads} threads, profiled: {n / sec / 1e6:.1f} M rows/s", flush=True)
        del os.environ["FLS_READ_PROFILE"]
        e.close()
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()
