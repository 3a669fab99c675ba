#!/usr/bin/env python3
"""End-to-end (PCIe-inclusive) scan rates, reported beside the HBM number:
  1. engine: fls_scan_* row groups decoded on the GPU and delivered into
     pinned host memory (H2D compressed batch -> decode -> D2H), all columns;
  2. DuckDB glue: read_fastlanes through the executor harness, i.e. the same
     plus the copy into 2048-row DataChunks and a checksum over every byte.
    python scripts/e2e.py [--scale 10]
"""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=10)
    a = ap.parse_args()
    import pkgload
    fl = pkgload.load()
    img = fl.gen_image("lineitem", a.scale)
    t = fl.Connection([0]).read_image(img)
    rows = 0
    byts = 0
    for _ in t.scan():  # warm (pins the image, allocates slots)
        break
    t0 = time.perf_counter()
    import ctypes as C
    out = fl.RowGroup()
    fl._check(fl.lib.fls_scan_begin(t.h, None, 0, t.nrowgroups))
    while fl._check(fl.lib.fls_scan_next(t.h, C.byref(out))) == 1:
        rows += out.nrows
        byts += out.nrows * 128
    dt = time.perf_counter() - t0
    print(f"engine scan -> pinned host: SF{a.scale:g} {rows} rows in {dt:.3f} s = {rows / dt / 1e6:.1f} M rows/s, "
          f"{byts / dt / 1e9:.1f} GB/s decoded delivered ({rows * 15 / dt / 1e9:.2f} G values/s)", flush=True)
    path = "/tmp/fls_e2e_lineitem.fls"
    img.write(path)
    from ext_harness import Ext
    e = Ext()
    ref = None
    for th in (1, 4, 8, 16):
        n, h, sec = e.scan_count("read_fastlanes", path, threads=th)
        ref = ref or (n, h)
        assert (n, h) == ref, "parallel scan changed the result"
        print(f"read_fastlanes DataChunks ({th} scan threads, copy + checksum): {n} rows in {sec:.3f} s = "
              f"{n / sec / 1e6:.1f} M rows/s", flush=True)
    for th in (1, 16):
        n2, h2, sec2 = e.scan_count("read_fastlanes", path, proj=[0, 5, 10], threads=th)
        print(f"read_fastlanes projected 3 cols, {th} threads: {n2 / sec2 / 1e6:.1f} M rows/s", flush=True)
    # pushed-down filters: rate over the table's rows
    q6 = [(10, ">= 1994-01-01"), (10, "< 1995-01-01"), (6, ">= 0.05"), (6, "<= 0.07"), (4, "< 24")]
    okey = [(0, ">= 1000000"), (0, "< 3000000")]
    for label, where, proj in (("Q6 (l_extendedprice, l_discount)", q6, [5, 6]),
                               ("l_orderkey range, all columns", okey, None)):
        for th in (1, 16):
            n3, _, sec3 = e.scan_count("read_fastlanes", path, proj=proj, threads=th, where=where)
            print(f"read_fastlanes WHERE {label}, {th} threads: {n3} rows selected of {rows}; "
                  f"{rows / sec3 / 1e6:.1f} M table rows/s ({sec3:.3f} s)", flush=True)
        n4, _, sec4 = e.scan_count("read_fastlanes", path, proj=sorted({c for c, _ in where} | set(proj or range(15))),
                                   threads=16)
        print(f"  same columns without pushdown (DuckDB would filter on the CPU after this): "
              f"{n4 / sec4 / 1e6:.1f} M rows/s ({sec4:.3f} s)", flush=True)
    e.close()


if __name__ == "__main__":
    main()
