#!/usr/bin/env python3
"""Engine scan (fls_scan_*: compressed batch H2D -> decode -> D2H into pinned
host memory, all columns) timed over several passes, for one package root
(A/B of two builds: --root <tree>).
    python scripts/scan_rate.py [--root .] [--scale 10] [--reps 5]"""
import argparse
import ctypes as C
import sys
import time
from pathlib import Path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", default=str(Path(__file__).resolve().parents[1]))
    ap.add_argument("--scale", type=float, default=10)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    sys.path.insert(0, a.root)
    import pkgload
    fl = pkgload.load()
    img = fl.gen_image("lineitem", a.scale)
    t = fl.Connection([0]).read_image(img)
    for _ in t.scan():
        break
    res = []
    for _ in range(a.reps):
        rows = 0
        t0 = time.perf_counter()
        out = fl.RowGroup()
        fl._check(fl.lib.fls_scan_begin(t.h, None, 0, t.nrowgroups))
        while fl._check(fl.lib.fls_scan_next(t.h, C.byref(out))) == 1:
            rows += out.nrows
        res.append(rows / (time.perf_counter() - t0) / 1e6)
    print(f"{a.root}: engine scan SF{a.scale:g} M rows/s per pass: {[round(x, 1) for x in res]}", flush=True)


if __name__ == "__main__":
    main()
