#!/usr/bin/env python3
"""Average per-launch PMC counters of one kernel from rocprofv3 --pmc passes
(counter_collection.csv files under the given directories).

    python scripts/pmc_summary.py <kernel-name-substring> <dir> [<dir> ...]
"""
import collections
import csv
import glob
import sys


def main():
    kern, dirs = sys.argv[1], sys.argv[2:]
    tot = collections.defaultdict(list)
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if kern in r["Kernel_Name"]:
                    tot[r["Counter_Name"]].append(float(r["Counter_Value"]))
    avg = {k: sum(v) / len(v) for k, v in tot.items()}
    wc = avg.get("SQ_WAVE_CYCLES", 1)
    for k, v in sorted(avg.items()):
        print(f"{k:24s} {v:14.4g}" + (f"  ({v / wc:.1%} of wave cycles)" if k.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""))
    if "SQ_LDS_BANK_CONFLICT" in avg and avg.get("SQ_LDS_IDX_ACTIVE"):
        print(f"bank conflict / LDS active  {avg['SQ_LDS_BANK_CONFLICT'] / avg['SQ_LDS_IDX_ACTIVE']:.3f}")


if __name__ == "__main__":
    main()
