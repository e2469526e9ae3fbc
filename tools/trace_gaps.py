#!/usr/bin/env python3
"""Diagnostic: steady-state duration of each ppe_* kernel and the idle gap before it, from a rocprofv3 kernel-trace
CSV (the last --last dispatches).

  python tools/trace_gaps.py gpurun_out/<tag>/kt_x/k_kernel_trace.csv [--last 48]
"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=48)
    a = ap.parse_args()
    ev = []
    for x in csv.DictReader(open(a.trace)):
        m = re.search(r"(ppe_\w+|df_\w+)", x["Kernel_Name"])
        if m:
            ev.append((int(x["Start_Timestamp"]), int(x["End_Timestamp"]), m.group(1)))
    ev.sort()
    last = ev[-a.last:]
    dur, gap = collections.defaultdict(list), collections.defaultdict(list)
    for i in range(1, len(last)):
        dur[last[i][2]].append((last[i][1] - last[i][0]) / 1e3)
        gap[last[i][2]].append((last[i][0] - last[i - 1][1]) / 1e3)
    tot = 0.0
    for k in dur:
        md, mg = sum(dur[k]) / len(dur[k]), sum(gap[k]) / len(gap[k])
        tot += md + mg
        print(f"{k:40s} n {len(dur[k]):3d}  duration {md:8.2f} us  gap before {mg:6.2f} us")
    print(f"sum of means (one of each): {tot:.2f} us")


if __name__ == "__main__":
    main()
