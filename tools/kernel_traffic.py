#!/usr/bin/env python3
"""Diagnostic: FETCH_SIZE / WRITE_SIZE per kernel name from two rocprofv3 --pmc passes (raw counter units, KiB as the
counters report them, summed over every dispatch of the kernel and divided by --calls), beside each kernel's average
duration from a --kernel-trace CSV of the same command.

  python tools/kernel_traffic.py --fetch f.csv --write w.csv [--trace k_kernel_trace.csv] --calls 8
"""
import argparse
import collections
import csv
import re


def sums(path, counter):
    out = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            m = re.search(r"(\w+_kernel\w*|\w+)(?=[<(])", r["Kernel_Name"])
            out[m.group(1) if m else r["Kernel_Name"][:40]] += float(r["Counter_Value"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--trace")
    ap.add_argument("--calls", type=int, default=1)
    a = ap.parse_args()
    f, w = sums(a.fetch, "FETCH_SIZE"), sums(a.write, "WRITE_SIZE")
    dur = collections.defaultdict(list)
    if a.trace:
        for r in csv.DictReader(open(a.trace)):
            m = re.search(r"(\w+_kernel\w*|\w+)(?=[<(])", r["Kernel_Name"])
            dur[m.group(1) if m else r["Kernel_Name"][:40]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k in sorted(set(f) | set(w), key=lambda k: -(f.get(k, 0) + w.get(k, 0))):
        d = dur.get(k)
        print(f"{k:40s} fetch {f.get(k, 0) / a.calls / 1024:9.2f} MiB  write {w.get(k, 0) / a.calls / 1024:9.2f} MiB"
              + (f"  avg {sum(d) / len(d):8.2f} us over {len(d)}" if d else ""))


if __name__ == "__main__":
    main()
