"""Per-kernel duration summary from a rocprofv3 SQLite output (run_results.db):
name, calls, average and total microseconds, optionally filtered by substrings.
Usage: python3 tools/kstats_db.py <db> [substr ...]"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
keys = sys.argv[2:]
rows = db.execute("select name, count(*), avg(duration)/1e3, sum(duration)/1e3 from kernels "
                  "group by name order by sum(duration) desc").fetchall()
for name, n, avg, tot in rows:
    if not keys or any(k in name for k in keys):
        print("%-60s %6d %10.1f us %12.1f us" % (name[:60], n, avg, tot))
