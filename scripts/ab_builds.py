#!/usr/bin/env python3
"""A/B of library builds that does not confuse a build with its buffers'
placement (round 6: the decode's speed depends on where the driver placed the
output buffers, profiles/r6/placement_*.txt; scripts/ab.py gave each build
one upload, so a build's time was its one placement's).  Every round uploads
the table again for every build (a new placement each time, chosen by the
product's own placement search, FLS_PLACEMENT_TRIES) and times a few launches;
the builds alternate, and the median over rounds compares them.

    python scripts/ab_builds.py --variants base,sc1 --workload lineitem_full --scale 12.5 --rounds 8
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
    spec = importlib.util.spec_from_file_location(f"fls_{name}", PKG / "__init__.py",
                                                  submodule_search_locations=[str(PKG)])
    m = importlib.util.module_from_spec(spec)
    sys.modules[f"fls_{name}"] = m
    spec.loader.exec_module(m)
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="base,sc1")
    ap.add_argument("--workload", default="lineitem_full")
    ap.add_argument("--scale", type=float, default=12.5)
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--verify", action="store_true", help="check every build's decode against the generator")
    a = ap.parse_args()
    import torch  # noqa: F401  (same runtime as the bench)
    names = a.variants.split(",")
    mods = {n: load_variant(n) for n in names}
    img = mods[names[0]].gen_image(a.workload, a.scale, a.rows)
    times = {n: [] for n in names}
    algo = None
    for r in range(a.rounds):
        order = names if r % 2 == 0 else names[::-1]
        for n in order:
            m = mods[n]
            t = m.Connection([0]).read_image(img)
            t.device_upload()
            t.device_decode()
            t.device_sync()
            for _ in range(a.reps):
                t.device_decode()
            st = t.device_sync()
            times[n].append(st.kernel_ms_total / st.timed_launches)
            algo = st.algo_bytes
            if a.verify and r == 0:
                bad = m.check_device_table(t, a.workload, a.scale, a.rows)
                print(f"{n}: verify {'OK' if not any(bad) else bad}", flush=True)
            t.close()
        print(f"round {r}: " + " ".join(f"{n} {times[n][-1]:.4f}" for n in names), flush=True)
    res = {n: {"median_ms": round(statistics.median(v), 4), "min_ms": round(min(v), 4), "max_ms": round(max(v), 4),
               "GBps": round(algo / statistics.median(v) / 1e6, 1)} for n, v in times.items()}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
