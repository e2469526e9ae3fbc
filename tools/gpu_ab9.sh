# box-matched ceiling: the memory skeleton of C1's traffic, then C1 itself, in one call on one box
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 120 tools/calib/stream_calib2 > $O/skeleton.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_bench.py --config C1 --steps 32 --rounds 3 \
  --variant cur=packet-process-engine_amd/libppe_hip.so:api=batches,bpl=0 > $O/ab_C1.txt 2>&1 || exit 1
timeout -k 10 120 tools/calib/stream_calib2 > $O/skeleton2.txt 2>&1
