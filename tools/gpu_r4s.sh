# round 4: C3 with a wider jump root (10 / 12 bits of sip instead of 8: shallower subtrees, more blocks), outputs checked
set -o pipefail
L=packet-process-engine_amd
O=api=batches,bpl=0,outs=part
bash tools/gpu_ab.sh ${1:-r4s} C3 "base=$L/libppe_hip.so:$O" "j10=$L/libppe_hip.so:jump=10,$O" "j12=$L/libppe_hip.so:jump=12,$O" \
  -- --steps 20 --rounds 4 --check
