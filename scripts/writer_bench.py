#!/usr/bin/env python3
"""Write-path rates: the CPU FastLanes encoder behind
COPY ... TO (FORMAT fls) and fls_writer_*.

  1. C-ABI writer (ENC_AUTO), 1 and N column-parallel threads: lineitem
     columns handed over as arrays (what COPY's sink does per row group),
     encoded and assembled;
  2. the seeded workload encoder (fls_gen_image: generate + encode) on N threads;
  3. COPY (SELECT * FROM read_fastlanes(src)) TO dst (FORMAT fls) through the
     executor harness: GPU scan of the source + encode + write (needs a GPU).

    python scripts/writer_bench.py [--scale 1] [--threads 16] [--copy] [--gpu]
"""
import argparse
import os
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--copy", action="store_true")
    ap.add_argument("--copy-only", action="store_true", help="only the COPY leg")
    ap.add_argument("--workload", default="lineitem", help="lineitem | lineitem_full (l_comment FSST)")
    ap.add_argument("--gpu", action="store_true", help="also the writer with fls_writer_set_device(0)")
    ap.add_argument("--batch", type=int, default=8, help="row groups per fls_writer_add_rowgroups call (arm)")
    ap.add_argument("--arms", default="", help="COPY leg: interleaved env arms 'name:VAR=v,VAR2=v;name2:...'")
    ap.add_argument("--reps", type=int, default=1, help="COPY leg: rounds over the arms")
    a = ap.parse_args()
    import pkgload
    fl = pkgload.load()
    wl = a.workload
    n = fl.gen_nrows(wl, a.scale)
    img = fl.gen_image(wl, a.scale, nthreads=a.threads)
    if a.copy_only:
        return copy_leg(fl, a, img)
    t = fl.Connection([0]).read_image(img)
    sch = t.schema()
    cols = []
    raw = 0
    for c, (name, ty, w, s, ob) in enumerate(sch):
        if ty == fl.VARCHAR and fl.gen_dict_string(wl, c, 0) is None:  # l_comment: free text
            vals = [x.decode() for x in fl.gen_strings(wl, c, 0, n, a.scale)]
            raw += sum(len(x) for x in vals)
            cols.append((name, ty, vals, fl.ENC_AUTO, w, s))
        elif ty == fl.VARCHAR:
            codes = fl.gen_values(wl, c, 0, n, np.uint32, a.scale)
            words = []
            while (x := fl.gen_dict_string(wl, c, len(words))) is not None:
                words.append(x)
            vals = [words[k] for k in codes]
            raw += int(np.array([len(x) for x in words])[codes].sum())
            cols.append((name, ty, vals, fl.ENC_AUTO, w, s))
        else:
            v = fl.gen_values(wl, c, 0, n, fl.NP_DTYPE[ty], a.scale)
            raw += v.nbytes
            cols.append((name, ty, v, fl.ENC_AUTO, w, s))
    # marshal every row group's buffers first (what a COPY sink already holds),
    # then time only the C-ABI encode + assemble
    import ctypes as C
    lib = fl.lib
    parts = []
    for r0 in range(0, n, fl.ROWGROUP):
        r1 = min(n, r0 + fl.ROWGROUP)
        keep, data, offs = [], (C.c_void_p * len(cols))(), (C.c_void_p * len(cols))()
        for c, (name, ty, vals, *_rest) in enumerate(cols):
            if ty == fl.VARCHAR:
                sl = [x.encode() for x in vals[r0:r1]]
                o = np.zeros(len(sl) + 1, dtype=np.uint32)
                o[1:] = np.cumsum([len(x) for x in sl])
                buf = np.frombuffer(b"".join(sl), dtype=np.uint8).copy()
                keep += [o, buf]
                data[c], offs[c] = buf.ctypes.data, o.ctypes.data
            else:
                part = np.ascontiguousarray(vals[r0:r1])
                keep.append(part)
                data[c] = part.ctypes.data
        parts.append((r1 - r0, data, offs, keep))
    ref_bytes = None
    arms = [(th, -1, 1) for th in sorted({1, a.threads})] + [(a.threads, -1, a.batch)]
    if a.gpu:
        arms += [(a.threads, 0, 1), (a.threads, 0, a.batch)]
    for th, dev, batch in arms:
        w = lib.fls_writer_new(0)
        lib.fls_writer_set_threads.argtypes = [C.c_void_p, C.c_int]
        lib.fls_writer_set_threads(w, th)
        if dev >= 0:  # integer columns chosen (ENC_AUTO) and encoded on the GPU
            fl._check(lib.fls_writer_set_device(w, dev))
        for name, ty, vals, enc, wd, sc in cols:
            fl._check(lib.fls_writer_add_column(w, name.encode(), ty, wd, sc, enc))
        t0 = time.perf_counter()
        if batch == 1:
            for m, data, offs, _ in parts:
                fl._check(lib.fls_writer_add_rowgroup(w, m, data, offs))
        else:  # batch row groups per call: pointer arrays laid out row group by row group
            nc = len(cols)
            for b0 in range(0, len(parts), batch):
                grp = parts[b0:b0 + batch]
                rows = (C.c_uint32 * len(grp))(*[g[0] for g in grp])
                data = (C.c_void_p * (nc * len(grp)))()
                offs = (C.c_void_p * (nc * len(grp)))()
                for k, (_, d, o, _) in enumerate(grp):
                    for c in range(nc):
                        data[k * nc + c], offs[k * nc + c] = d[c], o[c]
                fl._check(lib.fls_writer_add_rowgroups(w, len(grp), rows, data, offs))
        p, ln = C.c_void_p(), C.c_uint64()
        fl._check(lib.fls_writer_finish_image(w, C.byref(p), C.byref(ln)))
        dt = time.perf_counter() - t0
        out = C.string_at(p, ln.value)
        same = ""
        if ref_bytes is None:
            ref_bytes = out
        else:
            same = ", bytes identical to the 1-thread CPU file" if out == ref_bytes else ", BYTES DIFFER"
        lib.fls_image_free(p)
        lib.fls_writer_free(w)
        where = (f"GPU {dev} + {th} threads" if dev >= 0 else f"{th} threads") + \
            (f", {batch} row groups per call" if batch > 1 else "")
        print(f"C-ABI writer (ENC_AUTO, {where}), lineitem SF{a.scale:g}: {n} rows x {len(cols)} cols in "
              f"{dt:.2f} s = {n / dt / 1e6:.2f} M rows/s, {raw / dt / 1e6:.0f} MB/s of input -> "
              f"{ln.value / 1e6:.0f} MB (ratio {raw / ln.value:.2f}){same}", flush=True)
    for th in sorted({1, a.threads}):
        t0 = time.perf_counter()
        g = fl.gen_image(wl, a.scale, nthreads=th)
        dt = time.perf_counter() - t0
        print(f"generate + encode (fls_gen_image), {th} threads: {n / dt / 1e6:.1f} M rows/s "
              f"({g.len / 1e6:.0f} MB in {dt:.2f} s)", flush=True)
    if a.copy:
        copy_leg(fl, a, img)


def copy_leg(fl, a, img):
    """COPY through the executor harness at 1 (ordered) and N (unordered)
    sink threads; with --arms, the arms' environments interleaved round by
    round on the same source file (same-box A/B), medians reported."""
    import statistics
    from ext_harness import Ext
    arms = [("default", {})]
    if a.arms:
        arms = []
        for spec in a.arms.split(";"):
            name, _, kv = spec.partition(":")
            arms.append((name, dict(x.split("=", 1) for x in kv.split(",") if x)))
    e = Ext()
    times = {}
    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "src.fls"), os.path.join(d, "dst.fls")
        img.write(src)
        for _ in range(max(1, a.reps)):
            for name, env in arms:
                saved = {k: os.environ.get(k) for k in env}
                os.environ.update(env)
                try:
                    for th in sorted({1, a.threads}):
                        t0 = time.perf_counter()
                        rows = e.copy("read_fastlanes", src, dst, fmt="fls", threads=th)
                        dt = time.perf_counter() - t0
                        times.setdefault((name, th), []).append(dt)
                        what = "ordered, one sink" if th == 1 else f"unordered, {th} sink threads"
                        print(f"COPY (SELECT * FROM read_fastlanes) TO (FORMAT fls), {what} [{name}]: {rows} rows "
                              f"in {dt:.2f} s = {rows / dt / 1e6:.2f} M rows/s", flush=True)
                finally:
                    for k, v in saved.items():
                        if v is None:
                            os.environ.pop(k, None)
                        else:
                            os.environ[k] = v
    e.close()
    if len(arms) > 1 or a.reps > 1:
        for (name, th), v in sorted(times.items()):
            print(f"median [{name}] {th} sink thread(s): {rows / statistics.median(v) / 1e6:.2f} M rows/s "
                  f"over {len(v)} runs", flush=True)


if __name__ == "__main__":
    main()
