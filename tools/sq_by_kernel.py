#!/usr/bin/env python3
"""Diagnostic: every SQ counter of a rocprofv3 --pmc CSV summed per kernel name and divided by --calls.

  python tools/sq_by_kernel.py gpurun_out/<tag>/sq_D1/k_counter_collection.csv --calls 8
"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--calls", type=int, default=1)
    a = ap.parse_args()
    t = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(a.csv)):
        m = re.search(r"(\w+)(?=[<(])", r["Kernel_Name"])
        t[m.group(1) if m else r["Kernel_Name"][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
    names = sorted({c for v in t.values() for c in v})
    for k, v in sorted(t.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        print(k)
        for c in names:
            print(f"   {c:22s} {v.get(c, 0) / a.calls:14.0f}")


if __name__ == "__main__":
    main()
