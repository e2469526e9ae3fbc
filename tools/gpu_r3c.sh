# round 3 A/B: block levels and compact leaves per config (one process per config, variants interleaved)
set -o pipefail
bash tools/gpu_ab.sh r3c C3 k3=packet-process-engine_amd/libppe_hip.so:api=batches,bpl=0,outs=part k2=packet-process-engine_amd/libppe_hip.so:E_PPE_BLOCK_LEVELS=2,api=batches,bpl=0,outs=part k3mt4=packet-process-engine_amd/libppe_hip_mt34.so:api=batches,bpl=0,outs=part -- --steps 20 --rounds 4 && \
bash tools/gpu_ab.sh r3c C4 k2c=packet-process-engine_amd/libppe_hip.so:api=batches,bpl=0,outs=part k2nc=packet-process-engine_amd/libppe_hip.so:E_PPE_COMPACT=0,api=batches,bpl=0,outs=part k3c=packet-process-engine_amd/libppe_hip.so:E_PPE_BLOCK_LEVELS=3,api=batches,bpl=0,outs=part -- --steps 20 --rounds 4 && \
bash tools/gpu_ab.sh r3c C2 k2c=packet-process-engine_amd/libppe_hip.so:api=batches,bpl=0,outs=part k2nc=packet-process-engine_amd/libppe_hip.so:E_PPE_COMPACT=0,api=batches,bpl=0,outs=part -- --steps 20 --rounds 4
