# C1 A/B: partition-list store in lane order through LDS (PPE_CMP_LDS) vs the permuted global store
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
D=packet-process-engine_amd
timeout -k 10 300 python -u tools/ab_bench.py --config C1 --steps 32 --rounds 8 --check \
  --variant cur=$D/libppe_hip.so:api=batches,bpl=0 --variant cmplds=$D/libppe_hip_cmplds.so:api=batches,bpl=0 \
  --variant nocmp=$D/libppe_hip_abl4.so:api=batches,bpl=0 > $O/ab_C1.txt 2>&1 || exit 1
