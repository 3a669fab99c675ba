#!/usr/bin/env python3
"""Does the main decode's speed depend on where its HBM buffers land?
(of two builds in one process the second-loaded one ran
~10 % faster; identical code, different buffers.)

One library, one generated image.  Each trial optionally allocates a pad of
P MiB on the device first (shifting where the table's input image and output
columns land), uploads the table, times the decode (HIP events, median of
rounds), prints every buffer address (FLS_DEBUG's upload trace, summarised),
then frees the table and the pad.  `dual` keeps two uploaded tables alive and
alternates them, as scripts/ab.py does with two builds.

    python scripts/placement_probe.py --scale 12.5 --trials none,pad:2,pad:1024,dual,none
"""
import argparse
import ctypes as C
import os
import re
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="lineitem_full")
    ap.add_argument("--scale", type=float, default=12.5)
    ap.add_argument("--trials", default="none,pad:2,pad:64,pad:1024,pad:12288,none,dual")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--sleep", type=float, default=0.0, help="idle seconds before each trial")
    ap.add_argument("--sels", default="all", help="column selections timed per trial: all, a-b ranges, c+d lists "
                    "(comma separated); e.g. all,0-14,15 splits lineitem_full into its main and FSST parts")
    ap.add_argument("--clock-files", default="", help="glob of sysfs files sampled every 2 ms during a trial "
                    "(e.g. /sys/class/drm/card*/device/pp_dpm_[msf]clk); their distinct values per trial are printed")
    a = ap.parse_args()
    import glob
    import threading
    import time
    cfiles = sorted(glob.glob(a.clock_files)) if a.clock_files else []
    seen = {}
    stop = threading.Event()

    def sampler():
        while not stop.is_set():
            for f in cfiles:
                try:
                    txt = open(f).read()
                except OSError:
                    continue
                cur = [ln for ln in txt.splitlines() if ln.rstrip().endswith("*")] or [txt.strip()[:80]]
                seen.setdefault(f, {}).setdefault(cur[0].strip(), 0)
                seen[f][cur[0].strip()] += 1
            time.sleep(0.002)

    def clocks():
        out = "; ".join(f"{Path(f).parent.parent.name}/{Path(f).name}: {v}" for f, v in sorted(seen.items()))
        seen.clear()
        return out
    if cfiles:
        threading.Thread(target=sampler, daemon=True).start()
    import torch  # noqa: F401  (same runtime as the bench)
    import pkgload
    fl = pkgload.load()
    img = fl.gen_image(a.workload, a.scale)
    conn = fl.Connection([0])

    def upload():
        # capture the engine's FLS_DEBUG placement lines (written to fd 2)
        os.environ["FLS_DEBUG"] = "1"
        r, w = os.pipe()
        saved = os.dup(2)
        os.dup2(w, 2)
        try:
            t = conn.read_image(img)
            t.device_upload()
        finally:
            os.dup2(saved, 2)
            os.close(w)
            os.close(saved)
            os.environ.pop("FLS_DEBUG", None)
        txt = os.read(r, 1 << 20).decode(errors="replace")
        os.close(r)
        addrs = [int(x, 16) for x in re.findall(r"(?:image|out) (0x[0-9a-f]+)", txt)]
        qs = [float(x) for x in re.findall(r"placement dev \d+ set \d+: .* q ([0-9.]+)", txt)]
        kept = re.findall(r"kept set (\d+)", txt)
        dms = [float(x) for x in re.findall(r"placement dev \d+ set \d+: .*?decode ([0-9.-]+) ms", txt)]
        upload.last = f"placement q {qs} decode {dms} kept {kept[0] if kept else '-'}"
        return t, addrs

    def parse_sel(c):
        if c == "all":
            return None
        if "-" in c:
            lo, hi = map(int, c.split("-"))
            return list(range(lo, hi + 1))
        return [int(x) for x in c.split("+")]
    sels = [parse_sel(c) for c in a.sels.split(",")]

    def timeit(tabs, sel=None):
        times = [[] for _ in tabs]
        for t in tabs:
            t.device_decode(sel)
            t.device_sync()
        for _ in range(a.rounds):
            for i, t in enumerate(tabs):
                for _ in range(a.reps):
                    t.device_decode(sel)
                st = t.device_sync()
                times[i].append(st.kernel_ms_total / st.timed_launches)
        return times

    def desc(addrs):
        img_a, outs = addrs[0], addrs[1:]
        m2 = sorted({x % (2 << 20) for x in outs})
        return (f"image {img_a:#x} out[0] {outs[0]:#x} .. out[-1] {outs[-1]:#x}; "
                f"out mod 2MiB {[hex(x) for x in m2][:4]}; out GiB offsets "
                f"{[round((x - outs[0]) / 2**30, 3) for x in outs]}")

    for trial in a.trials.split(","):
        if a.sleep:
            time.sleep(a.sleep)
        clocks() if cfiles else None
        if trial == "dual":
            ta, aa = upload()
            tb, ab = upload()
            ts = timeit([ta, tb])
            for nm, t, ad, v in (("dual-A", ta, aa, ts[0]), ("dual-B", tb, ab, ts[1])):
                print(f"{nm:10s} median {statistics.median(v):.4f} ms min {min(v):.4f} rounds {[round(x, 3) for x in v]} "
                      f"| {desc(ad)}", flush=True)
            if cfiles:
                print("   clocks:", clocks(), flush=True)
            ta.close()
            tb.close()
            continue
        if trial.startswith("bestof:"):
            # K uploads alive at once, each timed briefly; keep the fastest
            k = int(trial.split(":")[1])
            cands = [upload() for _ in range(k)]
            quick = []
            for t, _ in cands:
                t.device_decode()
                t.device_sync()
                for _ in range(3):
                    t.device_decode()
                st = t.device_sync()
                quick.append(st.kernel_ms_total / st.timed_launches)
            best = min(range(k), key=lambda i: quick[i])
            for i, (t, _) in enumerate(cands):
                if i != best:
                    t.close()
            t, ad = cands[best]
            v = timeit([t])[0]
            print(f"{trial:10s} median {statistics.median(v):.4f} ms min {min(v):.4f} rounds {[round(x, 3) for x in v]} "
                  f"| candidates {[round(x, 3) for x in quick]} kept {best} | {desc(ad)}", flush=True)
            t.close()
            continue
        pad = C.c_void_p()
        mb = int(trial.split(":")[1]) if trial.startswith("pad:") else 0
        if mb:
            fl._check(fl.lib.fls_device_alloc(0, mb << 20, C.byref(pad)))
        t, ad = upload()
        for sname, sel in zip(a.sels.split(","), sels):
            v = timeit([t], sel)[0]
            print(f"{trial:10s} [{sname}] median {statistics.median(v):.4f} ms min {min(v):.4f} rounds "
                  f"{[round(x, 3) for x in v]} | {upload.last} | pad {pad.value or 0:#x} | {desc(ad)}", flush=True)
        if cfiles:
            print("   clocks:", clocks(), flush=True)
        t.close()
        if mb:
            fl._check(fl.lib.fls_device_free(0, pad))


if __name__ == "__main__":
    main()
