#!/usr/bin/env python3
"""GPU chunk encoder rates (csrc/fls_encode.hip).

  1. device-resident: fls_encode_device over a column already in HBM (the
     kernel alone, HIP events); roofline = (T/8 bytes read + chunk bytes
     written) per launch / kernel time, against 8 TB/s;
  2. the writer over host columns (lineitem integer columns, explicit
     FFOR / DELTA): CPU threads vs fls_writer_set_device (staging, H2D, one
     launch per row group, D2H), output checked byte-identical.

    python scripts/encode_bench.py [--rows 1000000000] [--scale 10] [--reps 5]
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def device_case(fl, name, ty, enc, vals, reps):
    n = len(vals)
    d_in = fl.DeviceBuffer.from_array(vals)
    slot = fl.encode_slot_bytes(ty, enc)
    nrg = (n + fl.ROWGROUP - 1) // fl.ROWGROUP
    d_out = fl.DeviceBuffer(slot * nrg)
    fl.encode_device(0, ty, enc, d_in.ptr, n, d_out.ptr)  # warm-up
    ms = []
    for _ in range(reps):
        lens, k = fl.encode_device(0, ty, enc, d_in.ptr, n, d_out.ptr)
        ms.append(k)
    med = sorted(ms)[len(ms) // 2]
    out = sum(lens)
    algo = vals.nbytes + out
    gbs = algo / (med * 1e-3) / 1e9
    d_in.free()
    d_out.free()
    return {"case": name, "rows": n, "in_bytes": int(vals.nbytes), "out_bytes": int(out),
            "kernel_ms": round(med, 4), "values_per_s": n / (med * 1e-3), "algo_GBps": round(gbs, 1),
            "frac_of_8TBps": round(gbs / 8000.0, 3)}


def writer_case(fl, scale, threads):
    import ctypes as C
    wl = "lineitem"
    n = fl.gen_nrows(wl, scale)
    img = fl.gen_image(wl, scale, nthreads=threads)
    t = fl.Connection([0]).read_image(img)
    cols = []
    for c, (name, ty, w, s, ob) in enumerate(t.schema()):
        if ty == fl.VARCHAR:
            continue
        v = fl.gen_values(wl, c, 0, n, fl.NP_DTYPE[ty], scale)
        cols.append((name, ty, v, fl.ENC_DELTA if name == "l_orderkey" else fl.ENC_FFOR, w, s))
    raw = sum(v.nbytes for _, _, v, *_ in cols)
    lib = fl.lib
    lib.fls_writer_set_threads.argtypes = [C.c_void_p, C.c_int]
    res = {}
    for mode in ("cpu", "gpu"):
        w = lib.fls_writer_new(0)
        lib.fls_writer_set_threads(w, threads)
        if mode == "gpu":
            fl._check(lib.fls_writer_set_device(w, 0))
        for name, ty, v, enc, wd, sc in cols:
            fl._check(lib.fls_writer_add_column(w, name.encode(), ty, wd, sc, enc))
        parts = []
        for r0 in range(0, n, fl.ROWGROUP):
            r1 = min(n, r0 + fl.ROWGROUP)
            keep = [np.ascontiguousarray(v[r0:r1]) for _, _, v, *_ in cols]
            data = (C.c_void_p * len(cols))(*[k.ctypes.data for k in keep])
            parts.append((r1 - r0, data, keep))
        t0 = time.perf_counter()
        for m, data, _ in parts:
            fl._check(lib.fls_writer_add_rowgroup(w, m, data, None))
        p, ln = C.c_void_p(), C.c_uint64()
        fl._check(lib.fls_writer_finish_image(w, C.byref(p), C.byref(ln)))
        dt = time.perf_counter() - t0
        res[mode] = (dt, C.string_at(p, ln.value))
        lib.fls_image_free(p)
        lib.fls_writer_free(w)
    same = res["cpu"][1] == res["gpu"][1]
    return {"case": f"writer lineitem SF{scale:g}, {len(cols)} integer columns (FFOR, l_orderkey DELTA)",
            "rows": n, "input_MB": round(raw / 1e6), "cpu_threads": threads,
            "cpu_s": round(res["cpu"][0], 3), "cpu_Mrows_per_s": round(n / res["cpu"][0] / 1e6, 1),
            "gpu_s": round(res["gpu"][0], 3), "gpu_Mrows_per_s": round(n / res["gpu"][0] / 1e6, 1),
            "bytes_identical": same}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000_000)
    ap.add_argument("--scale", type=float, default=10.0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--no-writer", action="store_true", help="device-resident cases only")
    a = ap.parse_args()
    import pkgload
    fl = pkgload.load()
    n = a.rows
    cases = [
        ("c3 keys INT64 DELTA", fl.INT64, fl.ENC_DELTA, lambda: fl.gen_values("c3", 0, 0, n, np.int64, 1.0, n)),
        ("c1 values INT32 FFOR (W=7)", fl.INT32, fl.ENC_FFOR, lambda: fl.gen_values("c1", 0, 0, n, np.int32, 1.0, n)),
        ("c3 keys INT64 FFOR", fl.INT64, fl.ENC_FFOR, lambda: fl.gen_values("c3", 0, 0, n, np.int64, 1.0, n)),
    ]
    for name, ty, enc, gen in cases:
        vals = gen()
        print(json.dumps(device_case(fl, name, ty, enc, vals, a.reps)), flush=True)
        del vals
    if not a.no_writer:
        print(json.dumps(writer_case(fl, a.scale, a.threads)), flush=True)


if __name__ == "__main__":
    main()
