# round 4: D1 — the assembly launch's stash word, datagram count and plan row in one round of loads (pre), plus the
# scatter passes' histogram-row loads and the ranked kernels' tile-count loads unrolled (pu), plus the parse reading
# a frame's first 48 bytes in one round of dword loads (pv)
set -o pipefail
O=gpurun_out/${1:-r4y}
mkdir -p $O
L=packet-process-engine_amd
PPE_LIB=$L/libppe_hip_dfpv.so timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_defrag.py tests/test_gpu_mbuf.py > $O/pytest_defrag.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_defrag.py --variant head=$L/libppe_hip_dfhead.so --variant pre=$L/libppe_hip_dfpre.so \
  --variant pu=$L/libppe_hip_dfpu.so --variant pv=$L/libppe_hip_dfpv.so > $O/ab_defrag.txt 2>&1
