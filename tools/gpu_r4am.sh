# round 4: D1 assembly launch with the stashes moved to the waves past the datagram count (no wave does both)
set -o pipefail
O=gpurun_out/${1:-r4am}
mkdir -p $O
L=packet-process-engine_amd
PPE_LIB=$L/libppe_hip_dfsplit.so timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_defrag.py tests/test_gpu_mbuf.py > $O/pytest_defrag.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_defrag.py --variant prod=$L/libppe_hip.so --variant split=$L/libppe_hip_dfsplit.so \
  > $O/ab_defrag.txt 2>&1
