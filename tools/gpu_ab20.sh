# C3 leaf-cap depth sweep with direct records (PPE_LEAF_CAP_DEPTH, 0 = uncapped), one process each
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
L=packet-process-engine_amd/libppe_hip.so
run() {
  PPE_LEAF_CAP_DEPTH=$2 PPE_LEAF_CAP_N=2 timeout -k 10 300 python -u tools/ab_bench.py --config C3 --steps 32 --rounds 3 \
    --variant cur=$L:api=batches,bpl=0 > $O/ab_$1.txt 2>&1 || exit 1
  grep "kernel med" $O/ab_$1.txt | sed "s/^/$1 /" >> $O/summary.txt
}
run off 0 && run d8 8 && run d10 10 && run d12 12 && run d6 6 && run off_b 0
