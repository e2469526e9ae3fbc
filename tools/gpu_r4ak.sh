# round 4: D1 admission look-back with a bounded, sleeping spin (error word instead of an endless wait)
set -o pipefail
O=gpurun_out/${1:-r4ak}
mkdir -p $O
L=packet-process-engine_amd
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_defrag.py tests/test_gpu_mbuf.py > $O/pytest_defrag.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_defrag.py --variant head=$L/libppe_hip_dfhead.so --variant bounded=$L/libppe_hip.so \
  > $O/ab_defrag.txt 2>&1
