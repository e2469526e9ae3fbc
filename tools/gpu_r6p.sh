# round 6 diagnostic: the per-launch reader event's cost by its creation flags (PPE_AB_READER_EV_FLAGS):
# (the PPE_AB_* environment hooks this diagnostic used were removed once r6r replaced the per-launch event)
# 2 = DisableTiming (product), 536870914 = + DisableSystemFence, 1073741826 = + ReleaseToDevice, and no record at all
# (PPE_AB_NO_READER_EVENT=1); F1 bench lines, alternating processes, then an F1 kernel trace per setting
set -o pipefail
O=gpurun_out/r6p; mkdir -p $O
run() {  # name flags noev
  PPE_AB_READER_EV_FLAGS=$2 PPE_AB_NO_READER_EVENT=$3 timeout -k 10 300 python bench.py --config F1 --steps 20 --warmup 5 --no-cpu-baseline > $O/F1_$1_$4.json 2> $O/F1_$1_$4.err
}
for i in 1 2 3; do
  run ev 2 0 $i || exit 1
  run nosys 536870914 0 $i || exit 1
  run dev 1073741826 0 $i || exit 1
  run noev 2 1 $i || exit 1
done
for V in "nosys 536870914" "dev 1073741826"; do
  set -- $V
  PPE_AB_READER_EV_FLAGS=$2 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_$1 -o run --output-format csv -- python bench.py --config F1 --steps 16 --warmup 5 --no-cpu-baseline > $O/prof_$1.log 2>&1 || exit 1
done
for f in $O/*_[123].json; do echo $f $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" $f); done
for V in nosys dev; do python tools/f1_timed_stats.py $O/prof_$V/run_kernel_trace.csv --steps 16; done
