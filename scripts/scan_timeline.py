#!/usr/bin/env python3
"""Kernel timeline of a warm read_fastlanes query (rocprofv3 --kernel-trace of
scripts/cold_query.py --child): how busy the scan's D2H copy kernel keeps the
link, and how long copy kernels wait behind decode kernels.

    python scripts/scan_timeline.py kt_kernel_trace.csv [--gap-ms 5]

Queries are told apart by idle gaps of more than --gap-ms between dispatches;
per query: wall time from the first dispatch's start to the last one's end,
the union of host_copy_kernel intervals (link busy), the summed decode time,
and the copy time that overlapped a decode on another stream.
"""
import argparse
import csv


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", ""),
                         r.get("Stream_Id", "")))
    rows.sort()
    return rows


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap-ms", type=float, default=5)
    a = ap.parse_args()
    rows = load(a.trace)
    groups, cur = [], []
    for r in rows:
        if cur and r[0] - max(x[1] for x in cur[-8:]) > a.gap_ms * 1e6:
            groups.append(cur)
            cur = []
        cur.append(r)
    if cur:
        groups.append(cur)
    for i, g in enumerate(groups):
        copies = [(s, e) for s, e, n, *_ in g if "host_copy_kernel" in n]
        decodes = [(s, e) for s, e, n, *_ in g if "host_copy_kernel" not in n and "rocclr" not in n]
        if len(copies) < 10:
            continue
        t0, t1 = g[0][0], max(x[1] for x in g)
        wall = (t1 - t0) / 1e6
        busy = union(copies) / 1e6
        dec = sum(e - s for s, e in decodes) / 1e6
        # copy time during which some decode was running
        ov = 0
        for s, e in copies:
            for ds, de in decodes:
                lo, hi = max(s, ds), min(e, de)
                if hi > lo:
                    ov += hi - lo
        names = sorted({n.split("(")[0][-40:] for _, _, n, *_ in g if "host_copy_kernel" not in n})
        print(f"query {i}: wall {wall:.2f} ms, {len(copies)} copies busy {busy:.2f} ms ({busy / wall:.2f} of wall), "
              f"mean copy {busy / len(copies) * 1e3:.0f} us; {len(decodes)} decodes {dec:.2f} ms; "
              f"copy-decode overlap {ov / 1e6:.2f} ms; kernels {names}")


if __name__ == "__main__":
    main()
