# round 6: the split-image cut-list kernel (C3) compiled for 7 / 6 waves per SIMD (PPE_CUT_SPLIT_WAVES: fewer SGPR
# spills, 71 VGPRs) against the product, bench layout (part8), C3
set -o pipefail
O=gpurun_out/r6ad; mkdir -p $O
L=packet-process-engine_amd
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_bench.py --config C3 --rounds 7 --steps 32 --check \
  --variant base=$L/libppe_hip.so:outs=part8 --variant cs7=$L/libppe_hip_cs7.so:outs=part8 \
  --variant cs6=$L/libppe_hip_cs6.so:outs=part8 > $O/ab_C3.txt 2>&1 || exit 1
grep -h "kernel med\|identical\|differ" $O/ab_C3.txt
