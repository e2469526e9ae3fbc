# round 6 diagnostic: the image-reader event bound to the classify dispatch as its stop event (PPE_AB_READER_BIND=1,
# (the PPE_AB_* environment hooks this diagnostic used were removed once r6r replaced the per-launch event)
# no marker packet of its own), created with DisableTiming (2) or default flags (0), against the product's
# hipEventRecord after the launch and against no record at all; F1 lines alternating, then a kernel trace each
set -o pipefail
O=gpurun_out/r6q; mkdir -p $O
PPE_AB_READER_BIND=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flow.py > $O/pytest_bind.txt 2>&1 || exit 1
run() {  # name bind flags noev i
  PPE_AB_READER_BIND=$2 PPE_AB_READER_EV_FLAGS=$3 PPE_AB_NO_READER_EVENT=$4 timeout -k 10 300 python bench.py --config F1 --steps 20 --warmup 5 --no-cpu-baseline > $O/F1_$1_$5.json 2> $O/F1_$1_$5.err
}
for i in 1 2 3; do
  run ev 0 2 0 $i || exit 1
  run bind2 1 2 0 $i || exit 1
  run bind0 1 0 0 $i || exit 1
  run noev 0 2 1 $i || exit 1
done
for V in "bind2 2" "bind0 0"; do
  set -- $V
  PPE_AB_READER_BIND=1 PPE_AB_READER_EV_FLAGS=$2 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_$1 -o run --output-format csv -- python bench.py --config F1 --steps 16 --warmup 5 --no-cpu-baseline > $O/prof_$1.log 2>&1 || exit 1
done
for f in $O/*_[123].json; do echo $f $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" $f); done
for V in bind2 bind0; do python tools/f1_timed_stats.py $O/prof_$V/run_kernel_trace.csv --steps 16; done
tail -1 $O/pytest_bind.txt
