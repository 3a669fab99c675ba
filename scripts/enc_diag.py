#!/usr/bin/env python3
"""Encoder diagnosis: per column, GPU-written vs CPU-written single-column
images at a given size / row-group size, repeated; prints the columns that
differ, the first differing offsets and whether repeats agree.
    FLS_LIB=libflsgpu_x.so python scripts/enc_diag.py [--n 20000] [--rowgroup 4096]"""
import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--rowgroup", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--only", default="all", help="all | narrow (T <= 32) | wide (T = 64) columns in the mixed file")
    ap.add_argument("--mixed-only", action="store_true")
    a = ap.parse_args()
    import pkgload
    fl = pkgload.load()
    from test_encode import _columns
    cols = _columns(fl, a.n, np.random.default_rng(a.n))
    if a.only != "all":
        wide = {fl.INT64, fl.UINT64, fl.DECIMAL}
        cols = [c for c in cols if (c[1] in wide) == (a.only == "wide")]
    bad = 0
    for col in ([] if a.mixed_only else cols):
        cpu = fl.write_image([col], rowgroup=a.rowgroup).tobytes()
        outs = [fl.write_image([col], rowgroup=a.rowgroup, device=0).tobytes() for _ in range(a.reps)]
        diffs = []
        for o in outs:
            if o == cpu:
                diffs.append(None)
                continue
            x = np.frombuffer(cpu, np.uint8)
            y = np.frombuffer(o, np.uint8)
            m = min(len(x), len(y))
            d = np.nonzero(x[:m] != y[:m])[0]
            diffs.append((len(x), len(y), int(d.size), d[:8].tolist()))
        if any(diffs):
            bad += 1
            print(col[0], diffs, "repeats agree" if all(x == diffs[0] for x in diffs) else "REPEATS DIFFER")
    # the whole mixed file too; a differing one is localised: the first
    # differing byte offsets and the (column, row group) chunks whose decode
    # (oracle) differs from the CPU file's
    cpu_img = fl.write_image(cols, rowgroup=a.rowgroup)
    cpu = cpu_img.tobytes()
    same = []
    for _ in range(a.reps):
        g_img = fl.write_image(cols, rowgroup=a.rowgroup, device=0)
        g = g_img.tobytes()
        same.append(g == cpu)
        if g != cpu:
            from oracle import flsref as ref
            x, y = np.frombuffer(cpu, np.uint8), np.frombuffer(g, np.uint8)
            m = min(len(x), len(y))
            d = np.nonzero(x[:m] != y[:m])[0]
            rc, rg_ = ref.RefFile(cpu_img), ref.RefFile(g_img)
            badc = [(c, r) for c in range(rc.ncols) for r in range(rc.nrowgroups)
                    if not np.array_equal(rc.decode(c, r), rg_.decode(c, r))]
            print(f"  differs: sizes {len(x)}/{len(y)}, {d.size} bytes, first at {d[:6].tolist()}; "
                  f"chunks decoding differently (col, rg): {badc[:12]} ({len(badc)})", flush=True)
    print(f"n={a.n} rowgroup={a.rowgroup} only={a.only} ({len(cols)} columns): mixed file identical:", same,
          "columns differing alone:", bad)


if __name__ == "__main__":
    main()
