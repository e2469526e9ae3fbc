# round 3 A/B: packed multi-tile key state (pk) and compact records read inside the walk (recw) against the build
set -o pipefail
for C in C3 C4 C2; do
bash tools/gpu_ab.sh r3e $C cur=packet-process-engine_amd/libppe_hip.so:api=batches,bpl=0,outs=part pk=packet-process-engine_amd/libppe_hip_pk.so:api=batches,bpl=0,outs=part recw=packet-process-engine_amd/libppe_hip_recw.so:api=batches,bpl=0,outs=part -- --steps 20 --rounds 4 --check || exit 1
done
