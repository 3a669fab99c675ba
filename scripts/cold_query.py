#!/usr/bin/env python3
"""The file's first read_fastlanes query in a FRESH process (cold: pinned host
buffers, streams and the HBM image are made on the way), then warm queries,
at N threads (the cold 16-thread DataChunk query).  One
process per run, so arms (environment) alternate across processes:

    python scripts/cold_query.py --arms "hm:FLS_PIN_ARENA_MB=0;arena:FLS_PIN_ARENA_MB=8192" --runs 3
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def child(path, threads, warm):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tests"))
    from ext_harness import Ext
    e = Ext()
    n, sec = e.scan_rows("read_fastlanes", path, threads=threads)
    out = {"cold_rows_s": n / sec, "rows": n, "warm_rows_s": []}
    for _ in range(warm):
        n, sec = e.scan_rows("read_fastlanes", path, threads=threads)
        out["warm_rows_s"].append(n / sec)
    e.close()
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="lineitem_full")
    ap.add_argument("--scale", type=float, default=10)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--arms", default="default:")
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--warm", type=int, default=3)
    ap.add_argument("--child", default="")
    ap.add_argument("--gen-only", default="", help="write the workload's file to this path and exit")
    ap.add_argument("--profile", action="store_true",
                    help="FLS_SCAN_PROFILE / FLS_READ_PROFILE in the children; their phase tables are printed")
    a = ap.parse_args()
    if a.child:
        child(a.child, a.threads, a.warm)
        return
    sys.path.insert(0, str(ROOT))
    import pkgload
    fl = pkgload.load()
    img = fl.gen_image(a.workload, a.scale, 0, 0, None, a.threads)
    if a.gen_only:
        img.write(a.gen_only)
        img.close()
        return
    fd, path = tempfile.mkstemp(suffix=".fls", dir=os.environ.get("TMPDIR", "/tmp"))
    os.close(fd)
    img.write(path)
    img.close()
    arms = []
    for spec in a.arms.split(";"):
        name, _, kv = spec.partition(":")
        arms.append((name, dict(x.split("=", 1) for x in kv.split(",") if x)))
    res = {n: [] for n, _ in arms}
    try:
        for r in range(a.runs):
            for name, env in arms:
                penv = {**os.environ, **env}
                if a.profile:
                    penv.update({"FLS_SCAN_PROFILE": "1", "FLS_READ_PROFILE": "1"})
                p = subprocess.run([sys.executable, __file__, "--child", path, "--threads", str(a.threads),
                                    "--warm", str(a.warm)], env=penv, capture_output=True, text=True, timeout=300)
                if a.profile:
                    print(f"--- run {r} {name}: profile (stderr)\n" + "\n".join(
                        ln for ln in p.stderr.splitlines() if "amdgpu.ids" not in ln)[-6000:], flush=True)
                if p.returncode != 0:
                    print(p.stderr[-2000:], file=sys.stderr)
                    sys.exit(p.returncode)
                d = json.loads(p.stdout.strip().splitlines()[-1])
                res[name].append(d)
                print(f"run {r} {name}: cold {d['cold_rows_s'] / 1e6:.1f} M rows/s, warm "
                      f"{[round(x / 1e6, 1) for x in d['warm_rows_s']]}", flush=True)
    finally:
        os.unlink(path)
    for name, v in res.items():
        cold = sorted(x["cold_rows_s"] for x in v)
        print(f"arm {name}: cold median {cold[len(cold) // 2] / 1e6:.1f} M rows/s (all {[round(c / 1e6, 1) for c in cold]})")


if __name__ == "__main__":
    main()
