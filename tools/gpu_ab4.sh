set -o pipefail
O=gpurun_out/$1
mkdir -p $O
P=packet-process-engine_amd
for K in 20 32; do
timeout -k 10 400 python -u tools/ab_bench.py --config C1 --nbufs 8 --steps $K --rounds 4 --check \
  --variant g1=$P/libppe_hip.so:api=batches,bpl=0,groups=1 --variant g2=$P/libppe_hip.so:api=batches,bpl=0,groups=2 \
  --variant g4=$P/libppe_hip.so:api=batches,bpl=0,groups=4 --variant g8=$P/libppe_hip.so:api=batches,bpl=0,groups=8 \
  --variant g32=$P/libppe_hip.so:api=batches,bpl=0,groups=32 --variant b2=$P/libppe_hip.so:api=batches,bpl=2,groups=1 \
  > $O/ab_C1_K$K.txt 2>&1 || exit 1
done
