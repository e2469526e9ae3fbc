#!/usr/bin/env python3
"""Per-kernel summary (calls, average / total µs) of a rocprofv3 rocpd database (ROCm 7 default output), the same
columns as `rocprofv3 --stats`' kernel_stats.csv.  Usage: tools/rocpd_stats.py <results.db> [out.csv]"""
import csv
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    rows = db.execute("select name, count(*), avg(end - start) / 1000.0, sum(end - start) / 1000.0, "
                      "min(end - start) / 1000.0, max(end - start) / 1000.0 from kernels group by name "
                      "order by sum(end - start) desc").fetchall()
    total = sum(r[3] for r in rows) or 1.0
    out = csv.writer(open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout)
    out.writerow(["Name", "Calls", "AverageUs", "TotalUs", "MinUs", "MaxUs", "Percentage"])
    for name, n, avg, tot, mn, mx in rows:
        out.writerow([name, n, f"{avg:.3f}", f"{tot:.3f}", f"{mn:.3f}", f"{mx:.3f}", f"{100 * tot / total:.2f}"])


if __name__ == "__main__":
    main()
