# round 4: D1 admission in 1024- / 512-thread workgroups (64 / 128 look-back participants for 65,536 fragments)
set -o pipefail
O=gpurun_out/${1:-r4aj}
mkdir -p $O
L=packet-process-engine_amd
PPE_LIB=$L/libppe_hip_dfa1k.so timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_defrag.py tests/test_gpu_mbuf.py > $O/pytest_defrag.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_defrag.py --variant prod=$L/libppe_hip.so --variant a1k=$L/libppe_hip_dfa1k.so \
  --variant a512=$L/libppe_hip_dfa512.so > $O/ab_defrag.txt 2>&1
