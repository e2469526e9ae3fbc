# C3: depth-capped leaf lists (analysis knob PPE_LEAF_CAP_DEPTH / PPE_LEAF_CAP_N, read by the compiler at commit; the
# current kernel scans a leaf list serially), one process per setting, baseline first and last
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
L=packet-process-engine_amd/libppe_hip.so
run() {
  PPE_LEAF_CAP_DEPTH=$1 PPE_LEAF_CAP_N=$2 timeout -k 10 300 python -u tools/ab_bench.py --config C3 --steps 32 --rounds 3 \
    --variant cur=$L:api=batches,bpl=0 > $O/ab_C3_d$1_n$2.txt 2>&1 || exit 1
  grep "kernel med" $O/ab_C3_d$1_n$2.txt | sed "s/^/d$1 n$2 /" >> $O/summary.txt
}
run 0 1 && run 6 2 && run 6 4 && run 8 2 && run 8 4 && run 0 1
