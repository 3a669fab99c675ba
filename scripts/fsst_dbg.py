#!/usr/bin/env python3
"""Launch geometry (FLS_DEBUG) and kernel time of the FSST kernels on
l_comment; usage: FLS_DEBUG=1 python scripts/fsst_dbg.py [--scale 10]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

ap = argparse.ArgumentParser()
ap.add_argument("--scale", type=float, default=10)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
import pkgload  # noqa: E402
fl = pkgload.load()
img = fl.gen_image("lineitem_full", a.scale)
t = fl.Connection([0]).read_image(img)
t.device_upload()
for _ in range(a.reps):
    t.device_decode([15])
    st = t.device_sync()
    print(f"l_comment: {st.kernel_ms:.3f} ms", flush=True)
