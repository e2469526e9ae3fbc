#!/usr/bin/env python3
"""F1's timed region from a rocprofv3 --kernel-trace of bench.py's F1 run (the kernel-stats average
mixed the parity-sample and warm-up batches with the timed ones).  bench.py runs F1 as: the 4 parity-sample batches
(64k packets), W warm-up batches, then the K timed batches, each batch one flow classify dispatch
(ppe_classify_kernel<..., FLOW=true>) and one ppe_flow_post_kernel; since round 6 (r6u) K more batches follow the timed
region, with dispatch events (the classify kernel's own time for the bench line).  So the timed region's batches are
the K flow classify dispatches before the last K (--tail: the last K, for a bench.py from before r6u).

  f1_timed_stats.py <kernel_trace.csv> --steps K [--tail] [--out summary.txt]

Prints per-kernel mean / median / min / max over the timed dispatches, the gaps (classify end → post start,
post end → next classify start) and the batch period (classify start → next classify start)."""
import argparse
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--tail", action="store_true", help="the last K dispatches (bench.py before r6u)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    is_cls = lambda r: "ppe_classify_kernel" in r["Kernel_Name"] and (", true, false>" in r["Kernel_Name"] or "ELb1ELb0E" in r["Kernel_Name"])  # noqa: E731
    is_post = lambda r: "ppe_flow_post_kernel" in r["Kernel_Name"]  # noqa: E731
    idx = [i for i, r in enumerate(rows) if is_cls(r)]
    timed = idx[-a.steps:] if a.tail else idx[-2 * a.steps:-a.steps]
    cls, post, g1, g2, period = [], [], [], [], []
    for j, i in enumerate(timed):
        c = rows[i]
        c0, c1 = int(c["Start_Timestamp"]), int(c["End_Timestamp"])
        cls.append((c1 - c0) / 1e3)
        p = next((rows[k] for k in range(i + 1, len(rows)) if is_post(rows[k])), None)
        if p is not None:
            p0, p1 = int(p["Start_Timestamp"]), int(p["End_Timestamp"])
            post.append((p1 - p0) / 1e3)
            g1.append((p0 - c1) / 1e3)
            if j + 1 < len(timed):
                n0 = int(rows[timed[j + 1]]["Start_Timestamp"])
                g2.append((n0 - p1) / 1e3)
                period.append((n0 - c0) / 1e3)
    lines = [f"F1 timed region: {len(timed)} of {len(idx)} flow classify dispatches "
             f"(dispatch ids {rows[timed[0]].get('Dispatch_Id')}..{rows[timed[-1]].get('Dispatch_Id')})"]

    def stat(name, v):
        if v:
            lines.append(f"  {name:28s} n {len(v):3d}  mean {statistics.mean(v):8.2f} us  median "
                         f"{statistics.median(v):8.2f}  min {min(v):8.2f}  max {max(v):8.2f}")
    stat("classify kernel", cls)
    stat("post kernel (finalize+update)", post)
    stat("gap classify -> post", g1)
    stat("gap post -> next classify", g2)
    stat("batch period", period)
    text = "\n".join(lines)
    print(text)
    if a.out:
        open(a.out, "w").write(text + "\n")


if __name__ == "__main__":
    main()
