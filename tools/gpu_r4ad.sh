# round 4: D1 empty datagram slots written by the place kernel's workgroups as coalesced stores (the assembly waves
# of empty slots only stash)
set -o pipefail
O=gpurun_out/${1:-r4ad}
mkdir -p $O
L=packet-process-engine_amd
PPE_LIB=$L/libppe_hip_dfzero.so timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_defrag.py tests/test_gpu_mbuf.py > $O/pytest_defrag.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_defrag.py --variant noidst=$L/libppe_hip_dfnoidst.so \
  --variant unroll=$L/libppe_hip_dfunroll.so --variant zero=$L/libppe_hip_dfzero.so > $O/ab_defrag.txt 2>&1
