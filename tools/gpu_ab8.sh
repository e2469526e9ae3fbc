# round-2 A/B: C1 single-tile kernel with the next tile's window prefetched into registers (6 / 7 / 8 waves per SIMD)
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
D=packet-process-engine_amd
timeout -k 10 300 python -u tools/ab_bench.py --config C1 --steps 32 --rounds 4 --check \
  --variant cur=$D/libppe_hip.so:api=batches,bpl=0 --variant pf6=$D/libppe_hip_pf6.so:api=batches,bpl=0 \
  --variant pf7=$D/libppe_hip_pf7.so:api=batches,bpl=0 --variant pf8=$D/libppe_hip_pf8.so:api=batches,bpl=0 > $O/ab_C1.txt 2>&1
