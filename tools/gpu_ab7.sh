# round-2 A/B: L2 residency of the classifier image against the packet stream (nt window loads, sc1 result stores)
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
D=packet-process-engine_amd
V="--variant cur=$D/libppe_hip.so:api=batches,bpl=0 --variant ntw=$D/libppe_hip_ntw.so:api=batches,bpl=0 --variant sc1=$D/libppe_hip_sc1.so:api=batches,bpl=0 --variant ntsc=$D/libppe_hip_ntsc.so:api=batches,bpl=0"
timeout -k 10 400 python -u tools/ab_bench.py --config C3 --steps 32 --rounds 3 --check $V > $O/ab_C3.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_bench.py --config C4 --steps 32 --rounds 3 --check $V > $O/ab_C4.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_bench.py --config C1 --steps 32 --rounds 3 --check \
  --variant cur=$D/libppe_hip.so:api=batches,bpl=0 --variant ntw2=$D/libppe_hip_ntw2.so:api=batches,bpl=0 \
  --variant sc1=$D/libppe_hip_sc1.so:api=batches,bpl=0 > $O/ab_C1.txt 2>&1 || exit 1
