# round 6: D1's process kernel with a register window of 8 / 4 (head + 7 / 3 group slots; groups past them take the
# linear member pass) against 16: 160 → 96 / 78 VGPRs.  Defrag GPU tests on each build, D1 lines alternating
set -o pipefail
O=gpurun_out/r6w; mkdir -p $O
L=packet-process-engine_amd
export TMPDIR=/tmp
for V in w8 w4; do
  PPE_LIB=$L/libppe_hip_$V.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_defrag.py > $O/pytest_$V.txt 2>&1 || exit 1
done
for i in 1 2 3; do
  for V in w16 w8 w4; do
    LIB=$L/libppe_hip_$V.so; [ $V = w16 ] && LIB=$L/libppe_hip.so
    PPE_LIB=$LIB timeout -k 10 300 python bench.py --config D1 --steps 20 --warmup 5 --no-cpu-baseline > $O/${V}_$i.json 2> $O/${V}_$i.err || exit 1
  done
done
PPE_LIB=$L/libppe_hip_w8.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_w8 -o run --output-format csv -- python bench.py --config D1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_w8.log 2>&1 || exit 1
for f in $O/*_[123].json; do echo $f $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" $f); done
grep -h "df_" $O/prof_w8/run_kernel_stats.csv | cut -c1-160
tail -n 1 $O/pytest_w8.txt $O/pytest_w4.txt
