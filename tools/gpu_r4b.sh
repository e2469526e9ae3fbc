# round 4: the producer / consumer walk (PF_PC) — its parity tests, a same-box A/B on C3, then the whole GPU suite
set -o pipefail
O=gpurun_out/${1:-r4b}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
    -k "c3_64k or every_kernel_variant" > $O/pytest_pc.txt 2>&1 && \
timeout -k 10 300 python -u tools/ab_bench.py --config C3 --check \
    --variant base=packet-process-engine_amd/libppe_hip.so:outs=part8,api=batches \
    --variant pc=packet-process-engine_amd/libppe_hip.so:outs=part8,api=batches,pipeline=6 > $O/ab_C3.txt 2>&1 && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
