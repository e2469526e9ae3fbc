set -o pipefail
O=gpurun_out/$1
mkdir -p $O
P=packet-process-engine_amd
for C in C3 C1; do
timeout -k 10 400 python -u tools/ab_bench.py --config $C --steps 32 --rounds 3 \
  --variant cur=$P/libppe_hip.so:api=batches,bpl=0 --variant now12=$P/libppe_hip_ld1.so:api=batches,bpl=0 \
  --variant noq2=$P/libppe_hip_ld2.so:api=batches,bpl=0 > $O/ab_$C.txt 2>&1 || exit 1
done
