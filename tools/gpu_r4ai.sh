# round 4: batch groups of waves (PPE_GROUPS 4 / 8 / 16) for C4 and C3, product build, outputs checked
set -o pipefail
L=packet-process-engine_amd
O=api=batches,bpl=0,outs=part
bash tools/gpu_ab.sh ${1:-r4ai} C4 "g8=$L/libppe_hip.so:$O" "g4=$L/libppe_hip.so:groups=4,$O" "g16=$L/libppe_hip.so:groups=16,$O" \
  -- --steps 20 --rounds 4 --check && \
bash tools/gpu_ab.sh ${1:-r4ai} C3 "g8=$L/libppe_hip.so:$O" "g4=$L/libppe_hip.so:groups=4,$O" "g16=$L/libppe_hip.so:groups=16,$O" \
  -- --steps 20 --rounds 4 --check
