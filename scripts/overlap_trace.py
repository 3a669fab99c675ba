#!/usr/bin/env python3
"""Decode lineitem_full a few times (target for rocprofv3 --kernel-trace):
shows whether the FSST kernels overlap the main decode kernel.
    python scripts/overlap_trace.py [--scale 100] [--reps 3]"""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=100)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import pkgload
    fl = pkgload.load()
    t = fl.Connection([0]).read_image(fl.gen_image("lineitem_full", a.scale))
    t.device_upload()
    for _ in range(a.reps):
        t.device_decode()
        st = t.device_sync()
        print(f"lineitem_full: {st.kernel_ms:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
