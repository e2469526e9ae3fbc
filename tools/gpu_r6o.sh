# round 6 diagnostic: what the per-launch image / ring reader event (hipEventRecord after every classify launch)
# (the PPE_AB_* environment hooks this diagnostic used were removed once r6r replaced the per-launch event)
# costs: F1 and C1 bench lines with PPE_AB_NO_READER_EVENT=1 (records skipped: unsafe for rule swaps, none here)
# against the product, alternating processes
set -o pipefail
O=gpurun_out/r6o; mkdir -p $O
for i in 1 2 3; do
  for V in ev noev; do
    E=0; [ $V = noev ] && E=1
    PPE_AB_NO_READER_EVENT=$E timeout -k 10 300 python bench.py --config F1 --steps 20 --warmup 5 --no-cpu-baseline > $O/F1_${V}_$i.json 2> $O/F1_${V}_$i.err || exit 1
  done
done
for i in 1 2; do
  for V in ev noev; do
    E=0; [ $V = noev ] && E=1
    PPE_AB_NO_READER_EVENT=$E timeout -k 10 300 python bench.py --config C1 --steps 20 --warmup 5 --no-cpu-baseline > $O/C1_${V}_$i.json 2> $O/C1_${V}_$i.err || exit 1
  done
done
PPE_AB_NO_READER_EVENT=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_noev -o run --output-format csv -- python bench.py --config F1 --steps 16 --warmup 5 --no-cpu-baseline > $O/prof_noev.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_ev -o run --output-format csv -- python bench.py --config F1 --steps 16 --warmup 5 --no-cpu-baseline > $O/prof_ev.log 2>&1 || exit 1
for f in $O/*_[123].json; do echo $f $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" $f); done
for V in ev noev; do python tools/f1_timed_stats.py $O/prof_$V/run_kernel_trace.csv --steps 16; done
