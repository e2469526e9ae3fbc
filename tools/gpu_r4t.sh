# round 4: D1 process kernel with windowed loads (three dependent rounds per FCB segment instead of one chain per
# fragment), the head reaching its FCB header through its parsed record; place hands the assembly the FCB record
set -o pipefail
O=gpurun_out/${1:-r4t}
mkdir -p $O
L=packet-process-engine_amd
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_defrag.py tests/test_gpu_mbuf.py > $O/pytest_defrag.txt 2>&1 || exit 1
timeout -k 10 240 python -u tools/ab_defrag.py --variant base=$L/libppe_hip_dfbase.so --variant win=$L/libppe_hip.so \
  > $O/ab_defrag.txt 2>&1
