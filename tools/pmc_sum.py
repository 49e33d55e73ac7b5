"""Average every counter per kernel over the passes under DIR (dev tool).
usage: pmc_sum.py DIR REGEX"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def main(root, pat):
    per = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        disp = defaultdict(lambda: defaultdict(float))
        names = {}
        for r in csv.DictReader(open(f)):
            d = (f, int(r["Dispatch_Id"]))
            names[d] = r["Kernel_Name"].split("(")[0].replace("void ", "")
            disp[d][r["Counter_Name"]] += float(r["Counter_Value"])
        for d, cs in disp.items():
            if re.search(pat, names[d]):
                for c, v in cs.items():
                    per[names[d]][c].append(v)
    for k, cs in sorted(per.items()):
        print(k[:90])
        for c, v in sorted(cs.items()):
            print(f"   {c:24s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main(*sys.argv[1:3])
