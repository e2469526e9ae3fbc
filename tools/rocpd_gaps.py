#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 rocpd database (the default output format when no --output-format is
given): calls, average / total duration, and the average gap before each kernel (start minus the previous
dispatch's end on the same queue), optionally restricted to names matching a substring.

  python tools/rocpd_gaps.py gpurun_out/r4u/kt/k_results.db [--match df_]
"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, queue_id from kernels order by start").fetchall()
    stats = defaultdict(lambda: [0, 0, 0, 0])   # calls, total ns, gap ns, gaps counted
    prev_end = {}
    for name, s, e, q in rows:
        short = name.replace("(anonymous namespace)::", "").split("(")[0][:60]
        st = stats[short]
        st[0] += 1
        st[1] += e - s
        if q in prev_end and s >= prev_end[q]:
            st[2] += s - prev_end[q]
            st[3] += 1
        prev_end[q] = e
    print(f"{'kernel':60s} {'calls':>6s} {'avg us':>9s} {'total us':>10s} {'gap us':>8s}")
    for k, (n, t, g, ng) in sorted(stats.items(), key=lambda kv: -kv[1][1]):
        if a.match and a.match not in k:
            continue
        print(f"{k:60s} {n:6d} {t / n / 1e3:9.2f} {t / 1e3:10.1f} {(g / ng / 1e3 if ng else 0):8.2f}")


if __name__ == "__main__":
    main()
