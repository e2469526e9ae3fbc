#!/bin/bash
# Round evidence for the stateless configs (run on the GPU box from the repo root):
#   bash tools/profile_round.sh <tag> "<configs>"     → gpurun_out/prof_<tag>/...
# per config: rocprofv3 --kernel-trace --stats of bench.py with every launch the timed shape (32-batch ring
# launches: --warmup 32 --steps 32), FETCH_SIZE and WRITE_SIZE in separate --pmc passes and TCC_HIT / TCC_MISS
# over tools/ring_run.py (the same launches, nothing else on the GPU), calibrated traffic JSON; for C1 also the SQ
# instruction mix.  Calibration: the memory skeleton of tools/calib/stream_calib.hip (known byte count).
set -o pipefail
T=${1:-r2}
CONFIGS=${2:-"C1 C2 C3 C4"}
O=gpurun_out/prof_$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
K=32
if [ ! -f $O/cal_fetch/cal_counter_collection.csv ]; then
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/cal_fetch -o cal -- tools/calib/stream_calib 1048576 4 > $O/cal_fetch.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/cal_write -o cal -- tools/calib/stream_calib 1048576 4 > $O/cal_write.log 2>&1 || exit 1
fi
for C in $CONFIGS; do
  B="bench.py --config $C --configs= --stateful= --warmup $K --steps $K --no-cpu-baseline --no-host-inclusive"
  R="tools/ring_run.py --config $C --batches $K --launches 3"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$C -o k -- python3 $B > $O/kt_$C.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_$C -o k -- python3 $R > $O/fetch_$C.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write_$C -o k -- python3 $R > $O/write_$C.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/tcc_$C -o k -- python3 $R > $O/tcc_$C.log 2>&1 || exit 1
  RP=$(grep -o "algorithmic_read_per_pkt [0-9.]*" $O/fetch_$C.log | awk '{print $2}')
  python3 tools/collect_traffic.py --config $C --fetch $O/fetch_$C/k_counter_collection.csv --write $O/write_$C/k_counter_collection.csv \
    --cal-fetch $O/cal_fetch/cal_counter_collection.csv --cal-write $O/cal_write/cal_counter_collection.csv \
    --n $((K * 1048576)) --read-per-pkt $RP --write-per-pkt 8 --out $O/${T}_traffic_$C.json > $O/traffic_$C.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $O/tcc_$C/k_counter_collection.csv --tiles $((K * 16384)) --min-us 50 > $O/tcc_$C.txt 2>&1
  if [ $C = C1 ] || [ $C = C3 ] || [ $C = C4 ]; then
    timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $O/sq_$C -o k -- python3 $R > $O/sq_$C.log 2>&1 || exit 1
    python3 tools/pmc_summary.py $O/sq_$C/k_counter_collection.csv --tiles $((K * 16384)) --min-us 50 > $O/sq_$C.txt 2>&1
  fi
  echo "profile $C done"
done
