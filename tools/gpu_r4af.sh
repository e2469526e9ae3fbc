# round 4: D1 radix sort with pass 1's histogram counted by pass 0's scatter (one launch fewer per call)
set -o pipefail
O=gpurun_out/${1:-r4af}
mkdir -p $O
L=packet-process-engine_amd
PPE_LIB=$L/libppe_hip_dfh2.so timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_defrag.py tests/test_gpu_mbuf.py > $O/pytest_defrag.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_defrag.py --variant prod=$L/libppe_hip.so --variant h2=$L/libppe_hip_dfh2.so \
  > $O/ab_defrag.txt 2>&1
