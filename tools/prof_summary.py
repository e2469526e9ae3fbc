"""Summarise rocprofv3 rocpd databases: per-kernel average duration and per-dispatch PMC counter sums."""
import sqlite3, sys, collections, glob

def summarize(db, kernel_like="ppe_classify_kernel"):
    con = sqlite3.connect(db)
    out = {}
    rows = con.execute("select name,total_calls,average from top_kernels").fetchall()
    out["kernels"] = rows
    rows = con.execute(f"select dispatch_id, counter_name, sum(value) from counters_collection "
                       f"where kernel_name like '%{kernel_like}%' group by dispatch_id, counter_name").fetchall()
    per = collections.defaultdict(list)
    for d, c, v in rows:
        per[c].append(v)
    out["counters"] = {c: sum(v) / len(v) for c, v in per.items()}
    out["ndisp"] = {c: len(v) for c, v in per.items()}
    return out

if __name__ == "__main__":
    for db in sys.argv[1:]:
        s = summarize(db)
        print(db)
        for k in s["kernels"][:3]:
            print("  kernel", k)
        for c, v in sorted(s["counters"].items()):
            print(f"  {c:28s} {v:16.1f}  (n={s['ndisp'][c]})")
