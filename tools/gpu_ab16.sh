# C1: batch groups per ring launch (PPE_GROUPS, read at context creation: one process per setting, 8 = default twice)
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
L=packet-process-engine_amd/libppe_hip.so
for g in 8 2 4 16 32 8; do
  PPE_GROUPS=$g timeout -k 10 200 python -u tools/ab_bench.py --config C1 --steps 32 --rounds 3 \
    --variant cur=$L:api=batches,bpl=0 > $O/ab_C1_g$g.txt 2>&1 || exit 1
  grep "kernel med" $O/ab_C1_g$g.txt | sed "s/^/G=$g /" >> $O/summary.txt
done
