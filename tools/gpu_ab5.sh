set -o pipefail
O=gpurun_out/$1
mkdir -p $O
P=packet-process-engine_amd
for C in C3 C4; do
timeout -k 10 500 python -u tools/ab_bench.py --config $C --steps 32 --rounds 3 --check \
  --variant cur=$P/libppe_hip.so:api=batches,bpl=0,outs=part \
  --variant m2w6b512=$P/libppe_hip_mt2w6.so:api=batches,bpl=0,outs=part,E_PPE_MT_BLOCK=512,E_PPE_MT_LDS=53000 \
  --variant m2w7b1024h=$P/libppe_hip_mt2w7.so:api=batches,bpl=0,outs=part,E_PPE_MT_LDS=80000 \
  --variant m3w5b256=$P/libppe_hip_mt3w5.so:api=batches,bpl=0,outs=part,E_PPE_MT_BLOCK=256,E_PPE_MT_LDS=32000 \
  --variant m4b512h=$P/libppe_hip.so:api=batches,bpl=0,outs=part,E_PPE_MT_BLOCK=512,E_PPE_MT_LDS=80000 > $O/ab_$C.txt 2>&1 || exit 1
done
