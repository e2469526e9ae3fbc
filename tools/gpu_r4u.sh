# round 4: D1 — windowed process loads (r4t), the stash in the assembly launch, and the assembly plan built by the
# place kernel (each assembly wave starts from one read); tests on the product build, in-process A/B, kernel trace
set -o pipefail
O=gpurun_out/${1:-r4u}
mkdir -p $O
L=packet-process-engine_amd
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_defrag.py tests/test_gpu_mbuf.py > $O/pytest_defrag.txt 2>&1 || exit 1
timeout -k 10 240 python -u tools/ab_defrag.py --variant base=$L/libppe_hip_dfbase.so \
  --variant fused=$L/libppe_hip_dfwin2.so --variant plan=$L/libppe_hip.so > $O/ab_defrag.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o k -- \
  python -u bench.py --config D1 --steps 20 --warmup 3 > $O/kt.log 2>&1
