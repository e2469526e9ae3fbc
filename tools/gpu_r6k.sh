# round 6: D1 datagram copy in one round per datagram (flat: each output dword is one lane's, whichever fragment
# holds it) against round 5's per-fragment copy (DF_FLAT=0, libppe_hip_seg.so) and flat builds of 2 / 8 dwords per lane per pass (the product: 4):
# the defrag GPU tests on the product build, then alternating bench.py D1 lines and one kernel trace per build
set -o pipefail
O=gpurun_out/r6k; mkdir -p $O
L=packet-process-engine_amd
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_defrag.py > $O/pytest.txt 2>&1 || exit 1
for i in 1 2 3; do
  for V in seg flat2 flat4 flat8; do
    LIB=$L/libppe_hip_$V.so; [ $V = flat4 ] && LIB=$L/libppe_hip.so
    PPE_LIB=$LIB timeout -k 10 300 python bench.py --config D1 --steps 20 --warmup 5 --no-cpu-baseline > $O/${V}_$i.json 2> $O/${V}_$i.err || exit 1
  done
done
for V in seg flat4; do
  LIB=$L/libppe_hip_$V.so; [ $V = flat4 ] && LIB=$L/libppe_hip.so
  PPE_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$V -o run -- python bench.py --config D1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_$V.log 2>&1 || exit 1
done
echo rc=0
