#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter_collection.csv per kernel (name prefix match) and print totals
and per-dispatch averages.  usage: tools/pmc_sum.py <counter_collection.csv> [name-substring ...]"""
import csv
import sys
from collections import defaultdict

path, pats = sys.argv[1], sys.argv[2:]
tot = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for r in csv.DictReader(open(path)):
    name = r.get("Kernel_Name", "")
    if pats and not any(p in name for p in pats):
        continue
    key = name[:60]
    tot[key][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[key].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
for k, c in tot.items():
    n = max(1, len(disp[k]))
    print(f"{k}  dispatches={n}")
    for cn, v in sorted(c.items()):
        print(f"   {cn:28s} total {v:16.0f}  per-dispatch {v / n:14.1f}")
