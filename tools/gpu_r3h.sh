# Round 3: software-pipelined multi-tile loop (PPE_MT_PF) at 2 / 3 / 4 tiles per wave against the round-2 loop,
# ring launches with the partition layout (the bench's shape), outputs checked against the first variant
set -o pipefail
L=packet-process-engine_amd
O="api=batches,bpl=0,outs=part"
for C in C4 C3 C2; do
  bash tools/gpu_ab.sh r3h $C base=$L/libppe_hip_base.so:$O pf4=$L/libppe_hip_pf4.so:$O pf3=$L/libppe_hip_pf3.so:$O \
    pf2=$L/libppe_hip_pf2.so:$O -- --steps 20 --rounds 4 --check || exit 1
done
