#!/usr/bin/env python3
"""HBM traffic per launch of the classify kernel from rocprofv3 PMC passes, calibrated on the memory-skeleton
kernel of tools/calib/stream_calib.hip (same access pattern, known byte count), as MI355X_MICROARCH.md's HBM section
prescribes (FETCH_SIZE is only calibrated for 16-B-per-lane coalesced reads; ours are row-per-lane).

  python tools/collect_traffic.py --fetch <bench fetch csv> --write <bench write csv> \
      --cal-fetch <calib fetch csv> --cal-write <calib write csv> --n 1048576 --out profiles/r1_traffic_C1.json
"""
import argparse
import re
import csv
import json
import statistics


def per_dispatch(path, kernel, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if re.search(kernel, r["Kernel_Name"]) and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--cal-fetch", required=True)
    ap.add_argument("--cal-write", required=True)
    ap.add_argument("--n", type=int, default=1 << 20, help="packets per classify dispatch")
    ap.add_argument("--cal-n", type=int, default=1 << 20, help="packets per calibration-kernel dispatch")
    ap.add_argument("--cal-kernel", default="k_row<true>")
    ap.add_argument("--read-per-pkt", type=float, default=68.0, help="algorithmic read bytes per packet (IMIX: "
                    "min(len, 64) + 4 averaged)")
    ap.add_argument("--write-per-pkt", type=float, default=8.0, help="algorithmic written bytes per packet (the "
                    "roofline's: verdict + flow hash + ACL hit, 8 packed / 12 as three words; the 1-B list entry is "
                    "traffic, not algorithmic)")
    ap.add_argument("--config", default="C1")
    ap.add_argument("--kernel", default="ppe_classify_kernel", help="dispatches whose kernel name matches this regular expression")
    ap.add_argument("--calls", type=int, default=0, help="sum every matching dispatch and divide by this many calls "
                    "(a multi-kernel call such as ppe_defrag) instead of the median per dispatch")
    ap.add_argument("--alg-bytes", type=float, default=0.0, help="algorithmic bytes per call (with --calls)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    n = a.n
    if a.calls:
        f = sum(per_dispatch(a.fetch, a.kernel, "FETCH_SIZE")) / a.calls
        w = sum(per_dispatch(a.write, a.kernel, "WRITE_SIZE")) / a.calls
    else:
        f = statistics.median(per_dispatch(a.fetch, a.kernel, "FETCH_SIZE"))
        w = statistics.median(per_dispatch(a.write, a.kernel, "WRITE_SIZE"))
    cf = statistics.median(per_dispatch(a.cal_fetch, a.cal_kernel, "FETCH_SIZE"))
    cw = statistics.median(per_dispatch(a.cal_write, a.cal_kernel, "WRITE_SIZE"))
    cal_rd, cal_wr = a.cal_n * 68, a.cal_n * 16  # skeleton: 64-B window + 4-B length read, 4 x 4-B results written
    kr, kw = cal_rd / cf, cal_wr / cw  # bytes per counter unit for this access pattern
    alg_rd, alg_wr = n * a.read_per_pkt, n * a.write_per_pkt
    if a.calls and a.alg_bytes:  # a whole call's algorithmic bytes (bench.py run_defrag's bytes_call)
        alg_rd, alg_wr = a.alg_bytes, 0.0
    out = {"config": a.config, "n_packets": n, "read_per_pkt": a.read_per_pkt, "write_per_pkt": a.write_per_pkt, "fetch_size_raw": f, "write_size_raw": w, "calib": {"fetch_raw": cf, "write_raw": cw,
           "bytes_per_fetch_unit": kr, "bytes_per_write_unit": kw, "kernel": a.cal_kernel},
           "read_bytes": f * kr, "write_bytes": w * kw, "traffic_bytes": f * kr + w * kw,
           "algorithmic_bytes": alg_rd + alg_wr,
           "traffic_over_algorithmic": (f * kr + w * kw) / (alg_rd + alg_wr)}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
