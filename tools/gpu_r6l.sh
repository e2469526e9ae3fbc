# round 6: D1 stash copy through buffer descriptors (branch-free: the stores no longer wait for each other; stash),
# plus the header words in one round and the segment head / tail bytes with the dwords (new), against
# the round-start build (libppe_hip_seg.so): defrag GPU tests on the product, alternating bench.py D1 lines, one
# kernel trace per build
set -o pipefail
O=gpurun_out/${1:-r6l}; mkdir -p $O
VARS=${2:-"seg stash new"}   # libppe_hip_<name>.so; new = the product build
PROF=${3:-"seg new"}
L=packet-process-engine_amd
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_defrag.py > $O/pytest.txt 2>&1 || exit 1
for i in 1 2 3; do
  for V in $VARS; do
    LIB=$L/libppe_hip_$V.so; [ $V = new ] && LIB=$L/libppe_hip.so
    PPE_LIB=$LIB timeout -k 10 300 python bench.py --config D1 --steps 20 --warmup 5 --no-cpu-baseline > $O/${V}_$i.json 2> $O/${V}_$i.err || exit 1
  done
done
for V in $PROF; do
  LIB=$L/libppe_hip_$V.so; [ $V = new ] && LIB=$L/libppe_hip.so
  PPE_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$V -o run -- python bench.py --config D1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_$V.log 2>&1 || exit 1
done
for f in $O/*_[123].json; do echo $f $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" $f); done
