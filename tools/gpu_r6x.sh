# round 6 diagnostic: F1's post launch (finalize + owner update) against its classify launch, per dispatch, from
# SQ and TCC counters (separate --pmc passes over bench.py's F1)
set -o pipefail
O=gpurun_out/r6x; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B="bench.py --config F1 --steps 8 --warmup 2 --no-cpu-baseline"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d $O/sq -o k -- python3 $B > $O/sq.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --kernel-trace --output-format csv -d $O/tcc -o k -- python3 $B > $O/tcc.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_INSTS_SMEM --kernel-trace --output-format csv -d $O/sq2 -o k -- python3 $B > $O/sq2.log 2>&1 || exit 1
python3 - <<'PY'
import csv, collections, re
for p in ("sq", "tcc", "sq2"):
    t = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
    for r in csv.DictReader(open(f"gpurun_out/r6x/{p}/k_counter_collection.csv")):
        k = r["Kernel_Name"]
        if "ppe_flow_post_kernel" in k: name = "post"
        elif "ppe_classify_kernel" in k and (", true, false>" in k or "ELb1ELb0E" in k): name = "classify_flow"
        else: continue
        t[name][r["Counter_Name"]] += float(r["Counter_Value"]); n[name].add(r["Dispatch_Id"])
    for name, v in t.items():
        print(p, name, "dispatches", len(n[name]))
        for c, x in sorted(v.items()): print(f"   {c:24s} {x / len(n[name]):16.0f}")
PY
