# round 4: D1 assembly copying a datagram's segments in two phases (loads, then stores; libppe_hip_asmpipe.so)
set -o pipefail
O=gpurun_out/${1:-r4r}
mkdir -p $O
L=packet-process-engine_amd
PPE_LIB=$L/libppe_hip_asmpipe.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_defrag.py tests/test_gpu_mbuf.py > $O/pytest_defrag_asmpipe.txt 2>&1 || exit 1
timeout -k 10 240 python -u tools/ab_defrag.py --variant base=$L/libppe_hip.so --variant pipe=$L/libppe_hip_asmpipe.so \
  > $O/ab_defrag.txt 2>&1
