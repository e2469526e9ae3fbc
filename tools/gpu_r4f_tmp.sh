set -o pipefail
O=gpurun_out/r4f; mkdir -p $O
L=packet-process-engine_amd
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || exit 1
bash tools/gpu_ab_configs.sh r4f "C1 C4 C2 C3" p8=$L/libppe_hip.so:api=batches,bpl=0,outs=part8 p32=$L/libppe_hip.so:api=batches,bpl=0,outs=part -- --steps 20 --rounds 4 || exit 1
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
