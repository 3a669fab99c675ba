#!/usr/bin/env python3
"""Per-wave timeline of one table decode launch (the timing build,
libflsgpu_trace.so: every decode_chunk call records its start / end from
s_memrealtime, 100 MHz, and every FSST vector its own -- the fused kernel's
main chunks and FSST vectors alike, shape enc 0xFE marking FSST).  Answers where a launch loses time against its
steady-state rate: the ramp at the start, the drain after the queue runs dry,
and per-chunk durations by column shape.

    FLS_LIB=libflsgpu_trace.so python scripts/wave_trace.py --workload lineitem_full --scale 12.5 --cols 0-14
"""
import argparse
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

REC = np.dtype([("t0", "<u8"), ("t1", "<u8"), ("wave", "<u4"), ("vr", "<u4"), ("hw", "<u4"), ("xcc", "<u4"),
                ("shape", "<u4"), ("max_w", "<u4")])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="lineitem_full")
    ap.add_argument("--scale", type=float, default=12.5)
    ap.add_argument("--cols", default="0-14")
    ap.add_argument("--bin-us", type=float, default=20.0)
    ap.add_argument("--env", default="", help="VAR=v,VAR2=v set for the traced launch")
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "wave_trace.npz"))
    ap.add_argument("--from-npz", default="", help="analyse a saved trace (no GPU)")
    a = ap.parse_args()
    if a.from_npz:
        z = np.load(a.from_npz)
        analyse(a, z["rec"], float(z["kernel_ms"]), len(z["rec"]))
        return
    os.environ.setdefault("FLS_LIB", "libflsgpu_trace.so")
    for kv in filter(None, a.env.split(",")):
        k, v = kv.split("=", 1)
        os.environ[k] = v
    import torch  # noqa: F401
    import pkgload
    fl = pkgload.load()
    lib = fl.lib
    lib.fls_trace_reset.restype = C.c_int
    lib.fls_trace_read.restype = C.c_int64
    lib.fls_trace_read.argtypes = [C.c_void_p, C.c_uint32]
    lib.fls_trace_fsst_reset.restype = C.c_int
    lib.fls_trace_fsst_read.restype = C.c_int64
    lib.fls_trace_fsst_read.argtypes = [C.c_void_p, C.c_uint32]
    lo, hi = map(int, a.cols.split("-")) if "-" in a.cols else (int(a.cols), int(a.cols))
    sel = list(range(lo, hi + 1))
    img = fl.gen_image(a.workload, a.scale)
    t = fl.Connection([0]).read_image(img)
    t.device_upload()
    for _ in range(3):
        t.device_decode(sel)
    t.device_sync()
    lib.fls_trace_reset()
    lib.fls_trace_fsst_reset()
    t.device_decode(sel)
    st = t.device_sync()
    cap = 1 << 20
    parts = []
    n = 0
    for read in (lib.fls_trace_read, lib.fls_trace_fsst_read):  # fls_decode.hip's records, fls_fsst.hip's
        buf = np.zeros(cap, REC)
        k = read(buf.ctypes.data, cap)
        n += k
        parts.append(buf[:min(k, cap)])
    r = np.concatenate(parts)
    kernel_ms = st.kernel_ms_total / max(1, st.timed_launches)
    analyse(a, r, kernel_ms, n)
    Path(a.out).parent.mkdir(exist_ok=True)
    np.savez_compressed(a.out, rec=r, kernel_ms=kernel_ms)


def analyse(a, r, kernel_ms, n):
    t0 = r["t0"].min()
    s = (r["t0"] - t0) / 100.0  # us
    e = (r["t1"] - t0) / 100.0
    span = e.max()
    vb = r["vr"] & 0xFF
    ve = r["vr"] >> 8
    fsst = (r["shape"] & 0xFF) == 0xFE  # one FSST vector per record (vr = its index)
    nv = np.where(fsst, 1, np.minimum(ve, r["shape"] >> 24) - vb)
    ob = (r["shape"] >> 16) & 0xFF
    byt = nv * (1024.0 * ob + 128.0 * r["max_w"])
    waves = np.unique(r["wave"])
    print(f"records {n}  waves {len(waves)}  launch span {span:.1f} us  (HIP-event kernel {kernel_ms * 1e3:.1f} us)")
    print(f"bytes (out + packed est.) {byt.sum() / 1e9:.3f} GB  = {byt.sum() / span / 1e6:.0f} GB/s over the span")
    # per wave: first start, last end
    first = np.full(waves.max() + 1, np.inf)
    last = np.zeros(waves.max() + 1)
    np.minimum.at(first, r["wave"], s)
    np.maximum.at(last, r["wave"], e)
    first, last = first[waves], last[waves]
    busy = np.zeros(waves.max() + 1)
    np.add.at(busy, r["wave"], e - s)
    busy = busy[waves]
    q = [0, 1, 5, 25, 50, 75, 95, 99, 100]
    print("wave first start (us) pct", dict(zip(q, np.percentile(first, q).round(1))))
    print("wave last end   (us) pct", dict(zip(q, np.percentile(last, q).round(1))))
    print(f"wave busy fraction of span: mean {busy.mean() / span:.3f}; idle after last end: mean {(span - last).mean():.1f} us")
    # bandwidth timeline: each call's bytes spread evenly over [s, e)
    nb = int(np.ceil(span / a.bin_us))
    tl = np.zeros(nb)
    act = np.zeros(nb)
    edges = np.arange(nb + 1) * a.bin_us
    for i in range(len(r)):
        b0, b1 = s[i], e[i]
        k0, k1 = int(b0 // a.bin_us), min(nb - 1, int(b1 // a.bin_us))
        rate = byt[i] / max(b1 - b0, 1e-3)
        for k in range(k0, k1 + 1):
            ov = min(b1, edges[k + 1]) - max(b0, edges[k])
            if ov > 0:
                tl[k] += rate * ov
                act[k] += ov / a.bin_us
    print(f"timeline ({a.bin_us:.0f} us bins): GB/s, active waves")
    for k in range(nb):
        print(f"  {edges[k]:7.0f} {tl[k] / a.bin_us / 1e3:7.0f} {act[k]:7.0f}")
    # main chunks against FSST vectors (the fused kernel's two queues)
    if fsst.any():
        print("kind: records, bytes (GB), first start, last end (us), wave-us busy, waves")
        for name, m in (("main", ~fsst), ("fsst", fsst)):
            if m.any():
                print(f"  {name}: {m.sum():7d} {byt[m].sum() / 1e9:7.3f} {s[m].min():8.1f} {e[m].max():8.1f} "
                      f"{(e[m] - s[m]).sum():10.0f} {len(np.unique(r['wave'][m])):5d}")
        print(f"timeline by kind ({a.bin_us:.0f} us bins): main GB/s, main waves, fsst GB/s, fsst waves")
        for k in range(nb):
            row = []
            for m in (~fsst, fsst):
                g = 0.0
                w = 0.0
                for i in np.flatnonzero(m & (s < edges[k + 1]) & (e > edges[k])):
                    ov = min(e[i], edges[k + 1]) - max(s[i], edges[k])
                    g += byt[i] / max(e[i] - s[i], 1e-3) * ov
                    w += ov / a.bin_us
                row += [g / a.bin_us / 1e3, w]
            print(f"  {edges[k]:7.0f} {row[0]:7.0f} {row[1]:7.0f} {row[2]:7.0f} {row[3]:7.0f}")
    # per shape: duration per vector
    keys = np.unique(r["shape"] & 0xFFFFFF)
    print("per chunk shape (enc, T, ob): calls, vectors, us per call mean / p95, us per vector (mean)")
    for k in keys:
        m = (r["shape"] & 0xFFFFFF) == k
        d = e[m] - s[m]
        print(f"  enc {k & 0xFF} T {(k >> 8) & 0xFF:2d} ob {(k >> 16) & 0xFF:2d}: {m.sum():6d} {nv[m].sum():8d} "
              f"{d.mean():8.1f} {np.percentile(d, 95):8.1f} {d.sum() / max(1, nv[m].sum()):7.2f}")
    # calls ending in the last 10 % of the span
    late = e > 0.9 * span
    print(f"calls ending in the last 10 % of the span: {late.sum()}, started at (us) pct",
          dict(zip(q, np.percentile(s[late], q).round(1))) if late.any() else {})
    # XCD balance
    for x in np.unique(r["xcc"] & 0xF):
        m = (r["xcc"] & 0xF) == x
        print(f"  xcc {x}: calls {m.sum()}, bytes {byt[m].sum() / 1e9:.3f} GB, last end {e[m].max():.1f} us")


if __name__ == "__main__":
    main()
