# round 4: D1 process kernel holding the chain's last word 0 in a register (appends read no LDS)
set -o pipefail
O=gpurun_out/${1:-r4ae}
mkdir -p $O
L=packet-process-engine_amd
PPE_LIB=$L/libppe_hip_dflast.so timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_defrag.py tests/test_gpu_mbuf.py > $O/pytest_defrag.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_defrag.py --variant zero=$L/libppe_hip_dfzero.so \
  --variant last=$L/libppe_hip_dflast.so > $O/ab_defrag.txt 2>&1
