#!/usr/bin/env python3
"""Per-trial PMC counters of one kernel: the kernel's dispatches, in dispatch
order, are cut into consecutive groups of N (one placement_probe trial = 1 warm
+ rounds x reps launches) and each group's median per counter is printed.

    python scripts/pmc_trials.py <kernel-substring> <N> <dir> [<dir> ...]
"""
import collections
import csv
import glob
import statistics
import sys


def main():
    kern, n, dirs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    per = collections.defaultdict(dict)  # dispatch id -> counter -> value
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if kern in r["Kernel_Name"]:
                    did = int(r["Dispatch_Id"])
                    per[did][r["Counter_Name"]] = per[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(per)
    names = sorted({k for v in per.values() for k in v})
    print("trial " + " ".join(f"{k:>32s}" for k in names))
    for t in range(0, len(ids), n):
        grp = ids[t:t + n]
        print(f"{t // n:5d} " + " ".join(f"{statistics.median(per[i].get(k, 0) for i in grp):32.5g}" for k in names))


if __name__ == "__main__":
    main()
