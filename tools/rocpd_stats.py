#!/usr/bin/env python3
"""rocprofv3 SQLite output (run_results.db) -> the --stats kernel_stats.csv columns.
Usage: python tools/rocpd_stats.py <run_results.db> <out.csv>"""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows)
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for n, k, s, a, lo, hi in rows:
            w.writerow([n, k, s, a, round(100.0 * s / tot, 2), lo, hi, 0.0])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
