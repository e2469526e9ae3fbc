# Round 3: GPU suite, then an A/B of the product against libppe_hip_bl.so (R3K = output tag)

set -o pipefail
O=gpurun_out/${R3K:-r3k}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || exit 1
L=packet-process-engine_amd
A="api=batches,bpl=0,outs=part"
for C in C4 C3 C2; do
  bash tools/gpu_ab.sh ${R3K:-r3k} $C new=$L/libppe_hip.so:$A old=$L/libppe_hip_bl.so:$A -- --steps 20 --rounds 4 --check || exit 1
done
