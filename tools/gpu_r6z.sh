# round 6: D1's place kernel walking the chain in rounds of 8 / 4 entries (DF_PLACE_H; the product: 8) instead of
# all 16 at once (144 → 99 / 60 VGPRs, 3 → 4 / 8 waves per SIMD).  Defrag GPU tests on each, D1 lines alternating,
# one kernel trace of the product
set -o pipefail
O=gpurun_out/r6z; mkdir -p $O
L=packet-process-engine_amd
export TMPDIR=/tmp
for V in h8 h4; do
  LIB=$L/libppe_hip_$V.so; [ $V = h8 ] && LIB=$L/libppe_hip.so
  PPE_LIB=$LIB timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_defrag.py > $O/pytest_$V.txt 2>&1 || exit 1
done
for i in 1 2 3; do
  for V in h16 h8 h4; do
    LIB=$L/libppe_hip_$V.so; [ $V = h8 ] && LIB=$L/libppe_hip.so
    PPE_LIB=$LIB timeout -k 10 300 python bench.py --config D1 --steps 20 --warmup 5 --no-cpu-baseline > $O/${V}_$i.json 2> $O/${V}_$i.err || exit 1
  done
done
for V in h8 h4; do
  LIB=$L/libppe_hip_$V.so; [ $V = h8 ] && LIB=$L/libppe_hip.so
  PPE_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$V -o run --output-format csv -- python bench.py --config D1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_$V.log 2>&1 || exit 1
done
for f in $O/*_[123].json; do echo $f $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" $f); done
for V in h8 h4; do echo $V; grep -h "df_place\|df_assemble" $O/prof_$V/run_kernel_stats.csv | cut -d, -f1-4; done
tail -n 1 $O/pytest_h8.txt $O/pytest_h4.txt
