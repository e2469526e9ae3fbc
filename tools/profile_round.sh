#!/bin/bash
# Collect the round's rocprofv3 evidence for the C1 bench (run on the GPU box, from the repo root):
#   kernel-trace stats, FETCH_SIZE / WRITE_SIZE passes (separate, kernel-trace only) for the bench and for the
#   memory-skeleton calibration kernel, SQ instruction-mix counters, and the calibrated traffic summary.
#   usage: bash tools/profile_round.sh r1      → gpurun_out/prof_r1/...
set -e
R=${1:-r1}
O=gpurun_out/prof_$R
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="bench.py --steps 48 --warmup 8 --no-cpu-baseline --no-host-inclusive"
P="bench.py --steps 16 --warmup 8 --no-cpu-baseline --no-host-inclusive"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o c1 -- python3 $B > $O/kt.log 2>&1
# the same bench with every launch on one stream (no overlap): kernel durations comparable with roofline.kernel_avg_us
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt1 -o c1 -- python3 $B --streams 1 > $O/kt1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o c1 -- python3 $P > $O/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o c1 -- python3 $P > $O/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/cal_fetch -o cal -- tools/calib/stream_calib 1048576 4 > $O/cal_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/cal_write -o cal -- tools/calib/stream_calib 1048576 4 > $O/cal_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $O/sq -o c1 -- python3 $P > $O/sq.log 2>&1
python3 tools/collect_traffic.py --fetch $O/fetch/c1_counter_collection.csv --write $O/write/c1_counter_collection.csv \
  --cal-fetch $O/cal_fetch/cal_counter_collection.csv --cal-write $O/cal_write/cal_counter_collection.csv \
  --n $((2 * 1048576)) --out $O/${R}_traffic_C1.json > $O/traffic.log 2>&1
python3 tools/pmc_summary.py $O/sq/c1_counter_collection.csv --tiles $((2 * 16384)) > $O/sq_summary.txt 2>&1
echo profile done
