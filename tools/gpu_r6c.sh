# round 6: the value region's fixed cost (tools/region_overhead.py) and the cut-lookup A/B (C4, C2: libppe_hip_cut1 vs base)
set -o pipefail
O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 300 python -u tools/region_overhead.py --steps 32 64 128 256 --rounds 5 > $O/region.txt 2>&1 && \
timeout -k 10 300 python -u tools/ab_bench.py --config C4 --rounds 7 --steps 32 --check \
  --variant base=packet-process-engine_amd/libppe_hip.so --variant cut1=packet-process-engine_amd/libppe_hip_cut1.so > $O/ab_C4.txt 2>&1 && \
timeout -k 10 300 python -u tools/ab_bench.py --config C2 --rounds 7 --steps 32 --check \
  --variant base=packet-process-engine_amd/libppe_hip.so --variant cut1=packet-process-engine_amd/libppe_hip_cut1.so > $O/ab_C2.txt 2>&1
echo rc=$?
