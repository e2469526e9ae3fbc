# C1 ablation on one box (PPE_ABLATE bits: 1 ACL, 2 counters, 4 compaction, 8 hash; 15 all four) + the memory skeleton
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
D=packet-process-engine_amd
timeout -k 10 300 python -u tools/ab_bench.py --config C1 --steps 32 --rounds 3 \
  --variant cur=$D/libppe_hip.so:api=batches,bpl=0 --variant noacl=$D/libppe_hip_abl1.so:api=batches,bpl=0 \
  --variant nocnt=$D/libppe_hip_abl2.so:api=batches,bpl=0 --variant nocmp=$D/libppe_hip_abl4.so:api=batches,bpl=0 \
  --variant nohash=$D/libppe_hip_abl8.so:api=batches,bpl=0 --variant none=$D/libppe_hip_abl15.so:api=batches,bpl=0 > $O/ab_C1.txt 2>&1 || exit 1
timeout -k 10 120 tools/calib/stream_calib2 > $O/skeleton.txt 2>&1
