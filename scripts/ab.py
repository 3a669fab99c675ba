#!/usr/bin/env python3
"""Interleaved A/B of decode-kernel builds in ONE process (rule: perf deltas
come from interleaved rounds on one device).  Each variant is an in-tree
build libflsgpu_<name>.so (make -C duckdb-fastlane_amd variants ...), loaded
side by side; the same SF image is uploaded once per variant and launches
alternate A, B, A, B ...  Kernel time from HIP events per launch.

    python scripts/ab.py --variants base,noseq [--scale 100] [--rounds 7] [--cols all,0,8]

Caveat (round 5, profiles/r5/ab_prefetch_order_r6b.txt): of two DIFFERENT
builds in one process, the one loaded second decoded lineitem_full SF12.5
~10 % faster whatever its code (3.109 ms first, 2.74-2.81 ms second, in both
orders), while one build loaded twice measured the same (ab_same_build_twice_
r6c.txt).  Compare builds in both orders, each at the same load position.
"""
import argparse
import importlib.util
import json
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "duckdb-fastlane_amd"


def load_variant(name):
    os.environ["FLS_LIB"] = "libflsgpu.so" if name == "base" else f"libflsgpu_{name}.so"
    mod_name = f"fls_{name}"
    spec = importlib.util.spec_from_file_location(mod_name, PKG / "__init__.py", submodule_search_locations=[str(PKG)])
    m = importlib.util.module_from_spec(spec)
    sys.modules[mod_name] = m
    spec.loader.exec_module(m)
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="base,noseq")
    ap.add_argument("--workload", default="lineitem")
    ap.add_argument("--scale", type=float, default=100)
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cols", default="all")
    a = ap.parse_args()
    import torch  # noqa: F401  (same runtime as the bench)
    names = a.variants.split(",")
    mods = {n: load_variant(n) for n in names}
    base = mods[names[0]]
    img = base.gen_image(a.workload, a.scale, a.rows)
    tabs = {}
    for n, m in mods.items():
        t = m.Connection([0]).read_image(img)
        t.device_upload()
        tabs[n] = t
    sels = [None if c == "all" else [int(c)] for c in a.cols.split(",")]
    res = {}
    for sel in sels:
        key = "ALL" if sel is None else tabs[names[0]].schema()[sel[0]][0]
        times = {n: [] for n in names}
        for n in names:  # warm
            tabs[n].device_decode(sel)
            tabs[n].device_sync()
        for _ in range(a.rounds):
            for n in names:
                for _ in range(a.reps):
                    tabs[n].device_decode(sel)
                st = tabs[n].device_sync()
                times[n].append(st.kernel_ms_total / st.timed_launches)
        st = tabs[names[0]].device_sync()
        line = {n: {"median_ms": round(statistics.median(v), 4), "min_ms": round(min(v), 4),
                    "GBps": round(st.algo_bytes / statistics.median(v) / 1e6, 1)} for n, v in times.items()}
        res[key] = line
        print(key, json.dumps(line), flush=True)
    out = ROOT / "gpurun_out" / "ab.json"
    out.parent.mkdir(exist_ok=True)
    out.write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
