#!/usr/bin/env python3
"""Prints the mean per-dispatch value of every counter in a
tools/profile_pmc.sh output directory, per kernel."""
import collections
import csv
import os
import sys

d = sys.argv[1]
for sub in sorted(os.listdir(d)):
    f = os.path.join(d, sub, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"].split("(")[0][-40:], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(agg.items()):
        print(f"{sub:6s} {k:40s} {c:22s} {sum(v) / len(v):.4g}")
