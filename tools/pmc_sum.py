#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter_collection.csv values per counter over the
dispatches of the FSM kernel, averaged per dispatch.
usage: tools/pmc_sum.py <dir with pass*/pmc_counter_collection.csv> [kernel substring]"""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    ksub = sys.argv[2] if len(sys.argv) > 2 else "solve_kernel"
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            if ksub not in r.get("Kernel_Name", ""):
                continue
            n = r["Counter_Name"]
            tot[n] += float(r["Counter_Value"])
            disp[n].add((f, r.get("Dispatch_Id", r.get("Correlation_Id", ""))))
    for n in sorted(tot):
        d = max(1, len(disp[n]))
        print(f"{n:28s} per_dispatch {tot[n] / d:.6e}  (dispatches {d})")


if __name__ == "__main__":
    main()
