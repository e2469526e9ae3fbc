# round 6: (1) the iterative-ilp machine scheduler on the current kernels, C1 / C2 in-process A/B (9 / 5 rounds) and
# F1 lines; (2) F1 with the owner-computed update off (PPE_FLOW_OWNER=0: the post launch is finalize alone), traced,
# to size what an update overlapped with the next classify could save
set -o pipefail
O=gpurun_out/r6s; mkdir -p $O
L=packet-process-engine_amd
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_bench.py --config C1 --rounds 9 --steps 32 --check \
  --variant base=$L/libppe_hip.so --variant iter=$L/libppe_hip_iterativeilp.so > $O/ab_C1.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_bench.py --config C2 --rounds 5 --steps 32 --check \
  --variant base=$L/libppe_hip.so --variant iter=$L/libppe_hip_iterativeilp.so > $O/ab_C2.txt 2>&1 || exit 1
for i in 1 2; do
  for V in base iter; do
    LIB=$L/libppe_hip.so; [ $V = iter ] && LIB=$L/libppe_hip_iterativeilp.so
    PPE_LIB=$LIB timeout -k 10 300 python bench.py --config F1 --steps 20 --warmup 5 --no-cpu-baseline > $O/F1_${V}_$i.json 2> $O/F1_${V}_$i.err || exit 1
  done
done
PPE_FLOW_OWNER=0 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_noowner -o run --output-format csv -- python bench.py --config F1 --steps 16 --warmup 5 --no-cpu-baseline > $O/prof_noowner.log 2>&1 || exit 1
grep -h "kernel med" $O/ab_C*.txt
for f in $O/F1_*_[12].json; do echo $f $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" $f); done
python tools/f1_timed_stats.py $O/prof_noowner/run_kernel_trace.csv --steps 16
