#!/usr/bin/env python3
"""Decode only l_comment (FSST) of lineitem_full a few times: target for
rocprofv3 --pmc passes on fsst_kernel.   python scripts/fsst_prof.py [--scale 10]
[--cols 0-14]: other columns instead (0-14: the main decode alone)."""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=10)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cols", default="15")
    ap.add_argument("--workload", default="lineitem_full")
    a = ap.parse_args()
    lo, hi = map(int, a.cols.split("-")) if "-" in a.cols else (int(a.cols), int(a.cols))
    cols = list(range(lo, hi + 1))
    import pkgload
    fl = pkgload.load()
    t = fl.Connection([0]).read_image(fl.gen_image(a.workload, a.scale))
    t.device_upload()
    for _ in range(a.reps):
        t.device_decode(cols)
    st = t.device_sync()
    print(f"cols {a.cols}: {st.kernel_ms_total / st.timed_launches:.3f} ms per launch", flush=True)


if __name__ == "__main__":
    main()
