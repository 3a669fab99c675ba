#!/usr/bin/env python3
"""Interleaved A/B of runtime decode knobs on ONE table and ONE set of HBM
buffers (A/B across separately loaded builds also changes where the 88 GB of
buffers land, which moved identical builds by 2-6 %).  An arm is a set of
environment variables the engine reads per decode call (FLS_DECODE_POLICY).

    python scripts/ab_env.py --arms "queue:FLS_DECODE_POLICY=0" "static:FLS_DECODE_POLICY=1" [--cols all,0]
"""
import argparse
import json
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", nargs="+", required=True, help="name:VAR=val,VAR2=val")
    ap.add_argument("--workload", default="lineitem")
    ap.add_argument("--scale", type=float, default=100)
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cols", default="all")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip checking each arm's decoded columns against the generator")
    a = ap.parse_args()
    import torch  # noqa: F401  (same runtime as the bench)
    import pkgload
    fl = pkgload.load()
    arms = []
    for spec in a.arms:
        name, _, kv = spec.partition(":")
        env = dict(x.split("=", 1) for x in kv.split(",") if x)
        arms.append((name, env))
    img = fl.gen_image(a.workload, a.scale, a.rows)
    t = fl.Connection([0]).read_image(img)
    t.device_upload()
    # a selection: "all", one column, or columns joined by "+" ("0-14": a range)
    def parse_sel(c):
        if c == "all":
            return None
        if "-" in c:
            lo, hi = map(int, c.split("-"))
            return list(range(lo, hi + 1))
        return [int(x) for x in c.split("+")]
    sels = [parse_sel(c) for c in a.cols.split(",")]
    res = {}
    any_bad = False

    def run(env, sel, reps):
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            for _ in range(reps):
                t.device_decode(sel)
            return t.device_sync()
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v

    for sel in sels:
        key = "ALL" if sel is None else t.schema()[sel[0]][0] if len(sel) == 1 else f"cols{sel[0]}-{sel[-1]}"
        times = {n: [] for n, _ in arms}
        for n, env in arms:  # warm (and build each arm's descriptor order once)
            run(env, sel, 1)
        algo = None
        for _ in range(a.rounds):
            for n, env in arms:
                run(env, sel, 1)  # descriptor rebuild for this arm happens outside the timed launches
                st = run(env, sel, a.reps)
                times[n].append(st.kernel_ms_total / st.timed_launches)
                algo = st.algo_bytes
        line = {n: {"median_ms": round(statistics.median(v), 4), "min_ms": round(min(v), 4),
                    "GBps": round(algo / statistics.median(v) / 1e6, 1)} for n, v in times.items()}
        if not a.no_verify:  # every arm's output, bit-exact against the seeded generator (on the GPU)
            for n, env in arms:
                run(env, sel, 1)
                mism = fl.check_device_table(t, a.workload, a.scale, a.rows)
                bad = {c: m for c, m in enumerate(mism) if m and (sel is None or c in sel)}
                line[n]["verified"] = not bad
                if bad:
                    any_bad = True
                    print(f"{key} arm {n}: MISMATCHING rows per column {bad}", flush=True)
        res[key] = line
        print(key, json.dumps(line), flush=True)
    out = ROOT / "gpurun_out" / "ab_env.json"
    out.parent.mkdir(exist_ok=True)
    out.write_text(json.dumps(res, indent=1))
    sys.exit(3 if any_bad else 0)


if __name__ == "__main__":
    main()
