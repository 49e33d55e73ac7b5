"""Print a rocprofv3 kernel_stats.csv as a short table (dev tool)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
for r in rows[:n]:
    print(f"{r['Name'][:72]:72s} {r['Calls']:>6s} {float(r['AverageNs'])/1000:10.1f}us {float(r['Percentage']):6.2f}%")
