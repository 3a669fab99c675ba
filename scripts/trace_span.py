#!/usr/bin/env python3
"""Per-step decode spans from a rocprofv3 kernel trace (out_kernel_trace.csv,
from `rocpd2csv -i run_results.db`).

A table decode step is several grids on two streams (the main decode_kernel
and the FSST kernel overlapped, flsgpu.hip launch_all), so rocprof's
per-kernel average is not the step time.  A step here = a maximal group of
decode/FSST dispatches whose [start, end) intervals overlap or touch within
`gap` ns; its span (first start -> last end) is what bench.py's HIP-event
kernel_ms measures.

    python scripts/trace_span.py out_kernel_trace.csv [--gap 20000]
"""
import argparse
import re
import csv
import statistics


def steps(path, gap):
    ev = []
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if "decode_kernel" in k or "fsst_kernel" in k or "fsst_sp_kernel" in k:
            m = re.search(r"(fsst_sp_kernel|fsst_kernel<[^>]*>|decode_kernel)", k)
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) + f" g{r['Grid_Size_X']}"))
    ev.sort()
    groups = []
    for s, e, k in ev:
        if groups and s <= groups[-1]["end"] + gap:
            g = groups[-1]
            g["end"] = max(g["end"], e)
            g["kernels"].append((k, e - s))
        else:
            groups.append({"start": s, "end": e, "kernels": [(k, e - s)]})
    return groups


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap", type=int, default=20000, help="ns between dispatches of one step")
    a = ap.parse_args()
    g = steps(a.trace, a.gap)
    spans = [(x["end"] - x["start"]) / 1e6 for x in g]
    for i, x in enumerate(g):
        ks = ", ".join(f"{k} {d / 1e6:.3f}" for k, d in x["kernels"])
        print(f"step {i:3d}: span {spans[i]:8.3f} ms  [{ks}]")
    if spans:
        big = [s for s in spans if s > 0.5 * max(spans)]
        print(f"{len(spans)} steps; full-size steps {len(big)}: mean span {statistics.mean(big):.3f} ms, "
              f"median {statistics.median(big):.3f} ms, min {min(big):.3f}, max {max(big):.3f}")


if __name__ == "__main__":
    main()
