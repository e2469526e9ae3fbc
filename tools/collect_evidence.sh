#!/bin/bash
# Copy one evidence set from gpurun_out/ into profiles/ under its tag (run here, after gpurun merged the outputs):
#   bash tools/collect_evidence.sh TAG
# from gpurun_out/TAG (tools/gpu_final.sh) and gpurun_out/prof_TAG (tools/profile_round.sh, tools/profile_stateful.sh)
T=$1
G=gpurun_out/$T
P=gpurun_out/prof_$T
D=profiles
[ -f $G/pytest_gpu.txt ] && cp $G/pytest_gpu.txt $D/${T}_pytest_gpu.txt
[ -f $G/smoke.txt ] && cp $G/smoke.txt $D/${T}_smoke.txt
[ -s $G/bench.json ] && cp $G/bench.json $D/${T}_bench_default_line.json
for C in C1 C2 C3 C4 F1 D1; do
  [ -f $P/kt_$C/k_kernel_stats.csv ] && cp $P/kt_$C/k_kernel_stats.csv $D/${T}_${C}_kernel_stats.csv
  [ -f $P/kt_$C.log ] && grep '^{' $P/kt_$C.log > $D/${T}_${C}_bench_under_rocprof.jsonl
  [ -f $P/${T}_traffic_$C.json ] && cp $P/${T}_traffic_$C.json $D/${T}_traffic_$C.json
  [ -f $P/tcc_$C.txt ] && cp $P/tcc_$C.txt $D/${T}_${C}_tcc.txt
  [ -f $P/sq_$C.txt ] && cp $P/sq_$C.txt $D/${T}_${C}_sq_counters.txt
done
# F1: the timed region's dispatches only (tools/f1_timed_stats.py over the kernel trace)
[ -f $P/${T}_F1_timed.txt ] && cp $P/${T}_F1_timed.txt $D/${T}_F1_timed_region.txt
ls $D | grep "^${T}_"
