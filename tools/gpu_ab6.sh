set -o pipefail
O=gpurun_out/$1
mkdir -p $O
L=packet-process-engine_amd/libppe_hip.so
timeout -k 10 300 python -u tools/ab_bench.py --config C1 --steps 32 --rounds 3 --check \
  --variant cur=$L:api=batches,bpl=0 --variant mt=$L:api=batches,bpl=0,pipeline=3 > $O/ab_C1.txt 2>&1 || exit 1
timeout -k 10 500 python -u tools/ab_bench.py --config C3 --steps 32 --rounds 3 --check \
  --variant cur=$L:api=batches,bpl=0 --variant j10=$L:api=batches,bpl=0,jump=10 --variant j12=$L:api=batches,bpl=0,jump=12 \
  --variant j14=$L:api=batches,bpl=0,jump=14 > $O/ab_C3.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_bench.py --config C2 --steps 32 --rounds 3 --check \
  --variant cur=$L:api=batches,bpl=0 --variant j8=$L:api=batches,bpl=0,jump=8 --variant j12=$L:api=batches,bpl=0,jump=12 > $O/ab_C2.txt 2>&1 || exit 1
