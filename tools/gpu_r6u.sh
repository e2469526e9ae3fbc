# round 6: F1's value region without dispatch events (the classify kernel time from K more batches after it) against
# the previous bench.py (bench_prev.py, events on every timed classify launch): F1 lines alternating, then a trace
set -o pipefail
O=gpurun_out/r6u; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  for V in prev new; do
    B=bench.py; [ $V = prev ] && B=bench_prev.py
    timeout -k 10 300 python $B --config F1 --steps 20 --warmup 5 --no-cpu-baseline > $O/F1_${V}_$i.json 2> $O/F1_${V}_$i.err || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_new -o run --output-format csv -- python bench.py --config F1 --steps 16 --warmup 5 --no-cpu-baseline > $O/prof_new.log 2>&1 || exit 1
for f in $O/F1_*_[123].json; do echo $f $(python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_avg_us'], r['batch_frac'])" $f); done
python tools/f1_timed_stats.py $O/prof_new/run_kernel_trace.csv --steps 16
