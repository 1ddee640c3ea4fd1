#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter CSVs per kernel (and per dispatch count) for a quick read."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
agg = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in sorted(glob.glob(f"{root}/pass*/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for (k, c), v in sorted(agg.items()):
    if k.startswith("__amd"):
        continue
    n = len(disp[(k, c)])
    print(f"{k:16s} {c:24s} total {v:14.4g}  per-dispatch {v / n:14.4g}  (n={n})")
