#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV output (counter_collection.csv) for one kernel: mean counter value per dispatch,
plus per-wave / per-tile derived figures.  Usage: pmc_summary.py <csv>... [--kernel substr] [--tiles N]"""
import argparse
import csv
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--kernel", default="ppe_classify_kernel")
    ap.add_argument("--tiles", type=int, default=16384)
    ap.add_argument("--min-us", type=float, default=0.0, help="only dispatches at least this long")
    a = ap.parse_args()
    per = defaultdict(lambda: defaultdict(float))  # (file, dispatch) -> counter -> value
    dur = {}
    for f in a.csv:
        for r in csv.DictReader(open(f)):
            if a.kernel not in r["Kernel_Name"]:
                continue
            key = (f, r["Dispatch_Id"])
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    cnt = defaultdict(list)
    per = {k: v for k, v in per.items() if dur[k] >= a.min_us}
    dur = {k: dur[k] for k in per}
    for key, d in per.items():
        for k, v in d.items():
            cnt[k].append(v)
    print(f"kernel ~ {a.kernel}: {len(per)} dispatches, mean duration {statistics.mean(dur.values()):.2f} us")
    for k in sorted(cnt):
        m = statistics.mean(cnt[k])
        print(f"  {k:28s} {m:16.1f}   per tile {m / a.tiles:10.2f}")


if __name__ == "__main__":
    main()
