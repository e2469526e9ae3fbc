# C3 / C4 / C1 with the packet stream served on-die (2 resident 1M-packet buffers reused by a 32-batch launch: 136 MB,
# inside the Infinity Cache) against 32 distinct buffers (HBM): how much of each config's time is the HBM stream
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
L=packet-process-engine_amd/libppe_hip.so
for c in C3 C4 C1; do
  timeout -k 10 200 python -u tools/ab_bench.py --config $c --steps 32 --rounds 3 --reuse --nbufs 2 \
    --variant cur=$L:api=batches,bpl=0 > $O/ab_${c}_mall.txt 2>&1 || exit 1
  timeout -k 10 200 python -u tools/ab_bench.py --config $c --steps 32 --rounds 3 \
    --variant cur=$L:api=batches,bpl=0 > $O/ab_${c}_hbm.txt 2>&1 || exit 1
done
