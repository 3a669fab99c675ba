#!/usr/bin/env python3
"""Per-step decode spans from a rocprofv3 kernel trace (*_kernel_trace.csv).

A table decode step is one or several grids (the main decode_kernel and the
FSST kernels, serial or overlapped on two streams, or one fused_kernel;
flsgpu.hip launch_all), so rocprof's per-kernel average is not the step time.
Every step starts with the reset of its work-queue counters (a fill-buffer
dispatch in the trace), so a step here = the decode dispatches between two
such resets; its span (first decode start -> last decode end) is what
bench.py's HIP-event kernel_ms measures.  Without fill dispatches in the trace
(an older run), dispatches whose intervals overlap or lie within `gap` ns are
grouped instead.

    python scripts/trace_span.py kt_kernel_trace.csv [--algo-bytes 121.908e9] [--peak 8e12]
"""
import argparse
import csv
import re
import statistics

DECODE = re.compile(r"(fused_kernel<[^>]*>|fsst_sp_kernel|fsst_kernel<[^>]*>|decode_kernel(?:<[^>]*>)?)")
# the upload's placement-rating launches (the same kernels under their RATING
# instantiation): not steps
RATING = re.compile(r"(decode_kernel<true>|fused_kernel<[^>]*,\s*true>)")


def events(path):
    ev = []
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if RATING.search(k):
            continue
        m = DECODE.search(k)
        if m:
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) + f" g{r['Grid_Size_X']}"))
        elif "fill" in k.lower():
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), None))  # a queue reset: step start
    ev.sort()
    return ev


def steps(ev, gap):
    groups = []
    use_fill = any(k is None for _, _, k in ev)
    new_step = True
    for s, e, k in ev:
        if k is None:
            new_step = True
            continue
        if groups and (not new_step if use_fill else s <= groups[-1]["end"] + gap):
            g = groups[-1]
            g["end"] = max(g["end"], e)
            g["kernels"].append((k, e - s))
        else:
            groups.append({"start": s, "end": e, "kernels": [(k, e - s)]})
        new_step = False
    return groups


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap", type=int, default=20000, help="ns between dispatches of one step (no fill dispatches)")
    ap.add_argument("--algo-bytes", type=float, default=0.0, help="algorithmic bytes of one step (bench roofline)")
    ap.add_argument("--peak", type=float, default=8e12, help="HBM peak, bytes/s")
    a = ap.parse_args()
    g = steps(events(a.trace), a.gap)
    spans = [(x["end"] - x["start"]) / 1e6 for x in g]
    for i, x in enumerate(g):
        ks = ", ".join(f"{k} {d / 1e6:.3f}" for k, d in x["kernels"])
        print(f"step {i:3d}: span {spans[i]:8.3f} ms  [{ks}]")
    if spans:
        big = [s for s in spans if s > 0.5 * max(spans)]
        m = statistics.mean(big)
        print(f"{len(spans)} steps; full-size steps {len(big)}: mean span {m:.3f} ms, "
              f"median {statistics.median(big):.3f} ms, min {min(big):.3f}, max {max(big):.3f}")
        if a.algo_bytes > 0:
            bw = a.algo_bytes / (m / 1e3)
            print(f"roofline from the mean span: {a.algo_bytes / 1e9:.3f} GB / {m:.3f} ms = {bw / 1e9:.1f} GB/s "
                  f"= {bw / a.peak:.3f} of {a.peak / 1e12:g} TB/s")


if __name__ == "__main__":
    main()
