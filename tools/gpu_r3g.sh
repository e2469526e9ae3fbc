# Round 3: component ablation of the multi-tile kernel on C4 (LDS image) and C3 (split image), in-process A/B
set -o pipefail
L=packet-process-engine_amd
for C in C4 C3; do
  bash tools/gpu_ab.sh r3g $C full=$L/libppe_hip.so noacl=$L/libppe_hip_abl1.so nocnt=$L/libppe_hip_abl2.so \
    nocmp=$L/libppe_hip_abl4.so nohash=$L/libppe_hip_abl8.so none=$L/libppe_hip_abl15.so || exit 1
done
