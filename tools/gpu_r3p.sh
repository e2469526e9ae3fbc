# Round 3: single-tile block kernel (tuning pipeline 5: 8 waves/SIMD, whole block section in LDS, compact records
# from L2) against the multi-tile kernel on C4 / C2
set -o pipefail
for C in C4 C2; do
  bash tools/gpu_ab.sh r3p $C mt=packet-process-engine_amd/libppe_hip.so:api=batches,bpl=0,outs=part sblk=packet-process-engine_amd/libppe_hip.so:api=batches,bpl=0,outs=part,pipeline=5 -- --steps 20 --rounds 4 --check || exit 1
done
