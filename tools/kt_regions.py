#!/usr/bin/env python3
"""Per-region kernel durations of a rocprofv3 --kernel-trace run of bench.py (dispatch order: warmup W, value K,
roofline-timing K).  Shows what the kernel-stats average mixes: in the pipelined value region two launches overlap,
so each lasts longer than a launch of the one-stream timing region, whose average is roofline.kernel_avg_us.
  kt_regions.py <kernel_trace.csv> [--warmup 10] [--steps 50]"""
import argparse
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--kernel", default="ppe_classify_kernel")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.csv)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    t0 = [int(r["Start_Timestamp"]) for r in rows]
    t1 = [int(r["End_Timestamp"]) for r in rows]
    w, k = a.warmup, a.steps
    print(f"{len(d)} dispatches of {a.kernel}")
    for name, lo, hi in (("warmup", 0, w), ("value", w, w + k), ("timing", w + k, w + 2 * k)):
        seg = d[lo:hi]
        if not seg:
            continue
        span = (max(t1[lo:hi]) - min(t0[lo:hi])) / 1e3
        print(f"  {name:7s} {len(seg):4d} launches: mean {statistics.mean(seg):7.2f} us  median {statistics.median(seg):7.2f}"
              f"  min {min(seg):7.2f}  max {max(seg):7.2f}   first start -> last end {span:8.1f} us"
              f" = {span / len(seg):6.2f} us per launch")


if __name__ == "__main__":
    main()
