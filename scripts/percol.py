#!/usr/bin/env python3
"""Per-column decode roofline: kernel time and algorithmic GB/s of the fused
decode launch restricted to one column at a time, plus device copy / fill
references measured the same way (HIP events) on the same GPU.

    python scripts/percol.py [--workload lineitem] [--scale 10] [--reps 5]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="lineitem")
    ap.add_argument("--scale", type=float, default=10)
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    import pkgload
    fl = pkgload.load()
    img = fl.gen_image(a.workload, a.scale, a.rows)
    t = fl.Connection([0]).read_image(img)
    t.device_upload()
    res = {}
    sch = t.schema()
    for sel in [[c] for c in range(t.ncols)] + [None]:
        t.device_decode(sel)
        t.device_sync()
        for _ in range(a.reps):
            t.device_decode(sel)
        st = t.device_sync()
        ms = st.kernel_ms_total / st.timed_launches
        name = "ALL" if sel is None else sch[sel[0]][0]
        res[name] = {"ms": round(ms, 4), "GBps": round(st.algo_bytes / ms / 1e6, 1),
                     "values": int(st.values), "packed": int(st.packed_bytes), "meta": int(st.meta_bytes),
                     "out": int(st.out_bytes)}
        print(f"{name:18s} {ms:8.3f} ms  {st.algo_bytes / ms / 1e6:8.1f} GB/s  "
              f"bits/val {8 * st.packed_bytes / max(1, st.values):5.1f}  out B/val {st.out_bytes / max(1, st.values):4.1f}",
              flush=True)
    # references: device copy (read+write) and fill (write) of 8 GiB
    n = 1 << 30
    x = torch.empty(n, dtype=torch.int64, device="cuda")
    y = torch.empty_like(x)
    for name, fn, nbytes in [("torch copy 8GiB", lambda: y.copy_(x), 2 * 8 * n),
                             ("torch fill 8GiB", lambda: y.fill_(7), 8 * n)]:
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        res[name] = {"ms": round(ms, 3), "GBps": round(nbytes / ms / 1e6, 1)}
        print(f"{name:18s} {ms:8.3f} ms  {nbytes / ms / 1e6:8.1f} GB/s", flush=True)
    Path(ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / f"percol_{a.workload}.json").write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
