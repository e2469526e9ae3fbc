# round 4: D1 process kernel counting statuses with one LDS atomic per fragment instead of a register-array select
set -o pipefail
O=gpurun_out/${1:-r4ab}
mkdir -p $O
L=packet-process-engine_amd
PPE_LIB=$L/libppe_hip_dfnoidst.so timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_defrag.py tests/test_gpu_mbuf.py > $O/pytest_defrag.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_defrag.py --variant noid=$L/libppe_hip_dfnoid.so --variant noidst=$L/libppe_hip_dfnoidst.so \
  > $O/ab_defrag.txt 2>&1
