#!/usr/bin/env python3
"""Per-dispatch start/end (relative, ms) from a rocprofv3 kernel_trace.csv."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("fls::(anonymous namespace)::", "")
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - t0) / 1e6
    print(f"{name[:40]:40s} grid {r.get('Grid_Size', r.get('Grid_Size_X', '?')):>8s} "
          f"start {s:10.3f} end {e:10.3f} dur {e - s:8.3f} ms")
