#!/usr/bin/env python
"""Summarise tools/pmc.sh output: mean per-dispatch value of each counter (development tool)."""
import csv, glob, os, sys
from collections import defaultdict

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
kfilter = sys.argv[2] if len(sys.argv) > 2 else ""  # substring of the kernel name
acc = defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
    per = defaultdict(float)
    for row in csv.DictReader(open(f)):
        if kfilter and kfilter not in row.get("Kernel_Name", ""):
            continue
        per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    for (disp, name), v in per.items():
        acc[name].append(v)
for name in sorted(acc):
    v = acc[name]
    print(f"{name:28s} {sum(v)/len(v):16.4g}  (n={len(v)})")
