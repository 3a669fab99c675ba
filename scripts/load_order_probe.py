#!/usr/bin/env python3
"""Does the product decode run faster when another build's kernels were
loaded first?  (scripts/ab.py measured the second-loaded of two different
builds ~10 % faster at lineitem_full SF12.5, profiles/r5/ab_prefetch_order_r6b.txt.)

    python scripts/load_order_probe.py [--first libflsgpu_exp.so] [--scale 12.5]

Loads --first (if given) as its own package instance, decodes a small table
with it (its kernels run once), then times the product build's table decode."""
import argparse
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "scripts"))
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--first", default="")
    ap.add_argument("--scale", type=float, default=12.5)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch  # noqa: F401
    import ab
    if a.first:
        name = a.first.replace("libflsgpu_", "").replace(".so", "")
        m0 = ab.load_variant(name)
        t0 = m0.Connection([0]).read_image(m0.gen_image("lineitem_full", 0.1))
        t0.device_upload()
        t0.device_decode(None)
        t0.device_sync()
    m = ab.load_variant("base")
    t = m.Connection([0]).read_image(m.gen_image("lineitem_full", a.scale))
    t.device_upload()
    for _ in range(3):
        t.device_decode(None)
    t.device_sync()
    ms = []
    for _ in range(a.reps):
        t.device_decode(None)
        st = t.device_sync()
        ms.append(st.kernel_ms_total / st.timed_launches)
    print(f"first={a.first or '-'} scale={a.scale}: median {statistics.median(ms):.4f} ms, min {min(ms):.4f}", flush=True)


if __name__ == "__main__":
    main()
