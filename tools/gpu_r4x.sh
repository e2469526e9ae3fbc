# round 4: D1 process kernel with the chain's word 0 per position in registers (independent compares and selects)
# instead of a serial LDS walk over the store slots
set -o pipefail
O=gpurun_out/${1:-r4x}
mkdir -p $O
L=packet-process-engine_amd
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_defrag.py tests/test_gpu_mbuf.py > $O/pytest_defrag.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_defrag.py --variant head=$L/libppe_hip_dfhead.so --variant regs=$L/libppe_hip.so \
  > $O/ab_defrag.txt 2>&1
