# round 6: D1's admission and grouping reading an FCB slot's state and creator together (one round trip, not two)
# against the previous build: defrag + mbuf GPU tests, D1 lines alternating, a kernel trace of each

set -o pipefail
O=gpurun_out/r6ah; mkdir -p $O
L=packet-process-engine_amd
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_defrag.py tests/test_gpu_mbuf.py > $O/pytest.txt 2>&1 || exit 1
for i in 1 2 3; do
  for V in base new; do
    LIB=$L/libppe_hip_$V.so; [ $V = new ] && LIB=$L/libppe_hip.so
    PPE_LIB=$LIB timeout -k 10 300 python bench.py --config D1 --steps 20 --warmup 5 --no-cpu-baseline > $O/${V}_$i.json 2> $O/${V}_$i.err || exit 1
  done
done
for V in base new; do
  LIB=$L/libppe_hip_$V.so; [ $V = new ] && LIB=$L/libppe_hip.so
  PPE_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$V -o run --output-format csv -- python bench.py --config D1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_$V.log 2>&1 || exit 1
done
for f in $O/*_[123].json; do echo $f $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" $f); done
for V in base new; do echo $V; grep -h "df_admit\|df_group" $O/prof_$V/run_kernel_stats.csv | cut -d, -f1-4; done
tail -1 $O/pytest.txt
