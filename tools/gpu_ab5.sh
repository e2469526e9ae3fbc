set -o pipefail
O=gpurun_out/$1
mkdir -p $O
P=packet-process-engine_amd
timeout -k 10 600 python -u tools/ab_bench.py --config C1 --steps 32 --rounds 4 \
  --variant r1=$P/libppe_hip_r1.so:api=batches,bpl=2 --variant ring8=$P/libppe_hip.so:api=batches,bpl=0,groups=8 \
  --variant ring1=$P/libppe_hip.so:api=batches,bpl=0,groups=1 --variant b4g1=$P/libppe_hip.so:api=batches,bpl=4,groups=1 \
  --variant b4g4=$P/libppe_hip.so:api=batches,bpl=4,groups=4 --variant b8g8=$P/libppe_hip.so:api=batches,bpl=8,groups=8 \
  --variant b16g8=$P/libppe_hip.so:api=batches,bpl=16,groups=8 --variant b8g1=$P/libppe_hip.so:api=batches,bpl=8,groups=1 \
  > $O/ab_C1.txt 2>&1
