# round 4: PF_PC tuning — role balance and queue depth on C3, and where each role waits
set -o pipefail
O=gpurun_out/${1:-r4c}
mkdir -p $O
L=packet-process-engine_amd
timeout -k 10 200 python -u tools/pc_stats.py --lib $L/libppe_hip_pcstats.so --config C3 > $O/pc_stats_C3.txt 2>&1 && \
timeout -k 10 200 python -u tools/pc_stats.py --lib $L/libppe_hip_pcstats.so --config C4 > $O/pc_stats_C4.txt 2>&1 && \
timeout -k 10 400 python -u tools/ab_bench.py --config C3 --rounds 5 \
    --variant base=$L/libppe_hip.so:outs=part8,api=batches \
    --variant pc4=$L/libppe_hip.so:outs=part8,api=batches,pipeline=6 \
    --variant pc2=$L/libppe_hip_pc2.so:outs=part8,api=batches,pipeline=6 \
    --variant pc6=$L/libppe_hip_pc6.so:outs=part8,api=batches,pipeline=6 \
    --variant pc8=$L/libppe_hip_pc8.so:outs=part8,api=batches,pipeline=6 \
    --variant q16=$L/libppe_hip_q16.so:outs=part8,api=batches,pipeline=6 > $O/ab_C3.txt 2>&1
