#!/usr/bin/env python3
"""dev: mean per-dispatch counter values of the kernels whose name contains
PATTERN, from a rocprofv3 --pmc csv directory.  usage: pmc_sum.py DIR PATTERN"""
import csv
import glob
import os
import sys
from collections import defaultdict

d, pat = sys.argv[1], sys.argv[2]
files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
vals = defaultdict(lambda: defaultdict(list))
for f in files:
    with open(f) as fh:
        for r in csv.DictReader(fh):
            name = r.get("Kernel_Name", "")
            if pat not in name:
                continue
            key = name.split("(")[0][:70]
            vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"  {c:28s} n={len(v):3d} mean={sum(v) / len(v):.4g}")
