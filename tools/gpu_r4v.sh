# round 4: D1 — the claim's first CAS expecting EMPTY (claim), the admission's look-back without the tile-count
# launch (look), and the assembly copy at 8 dwords per lane per pass with the funnel partner shuffled from the next
# lane (u8: 7 waves per SIMD; u8w8: held to 8, 4 VGPRs spilled)
set -o pipefail
O=gpurun_out/${1:-r4v}
mkdir -p $O
L=packet-process-engine_amd
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_defrag.py tests/test_gpu_mbuf.py > $O/pytest_defrag.txt 2>&1 || exit 1
PPE_LIB=$L/libppe_hip_dfu8w8.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_defrag.py > $O/pytest_defrag_u8w8.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_defrag.py --variant fused=$L/libppe_hip_dfwin2.so \
  --variant claim=$L/libppe_hip_dfclaim.so --variant look=$L/libppe_hip_dflook.so --variant u8=$L/libppe_hip.so \
  --variant u8w8=$L/libppe_hip_dfu8w8.so > $O/ab_defrag.txt 2>&1
