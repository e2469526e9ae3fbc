# round 4: D1 — claim fused into the parse launch, the admission look-back 64 predecessors per round (wave 0), and
# the assembly copy at 8 vs 4 dwords per lane per pass (funnel partner shuffled), and the admission launch computing
# the group keys and the first radix histogram (adm, the product build); tests, A/B, kernel trace
set -o pipefail
O=gpurun_out/${1:-r4w}
mkdir -p $O
L=packet-process-engine_amd
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_defrag.py tests/test_gpu_mbuf.py > $O/pytest_defrag.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_defrag.py --variant claim=$L/libppe_hip_dfclaim.so \
  --variant look1=$L/libppe_hip_dfparse.so --variant look2=$L/libppe_hip_dflook2.so --variant u4=$L/libppe_hip_dfu4.so --variant adm=$L/libppe_hip.so \
  > $O/ab_defrag.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o k -- \
  python3 bench.py --config D1 --steps 20 --warmup 3 --no-cpu-baseline > $O/kt.log 2>&1
