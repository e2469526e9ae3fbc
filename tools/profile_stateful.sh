#!/bin/bash
# Round evidence for the stateful rows (run on the GPU box from the repo root):
#   bash tools/profile_stateful.sh <tag>     → gpurun_out/prof_<tag>/...
# F1 (flow table): rocprofv3 --kernel-trace --stats of bench.py --config F1, FETCH_SIZE and WRITE_SIZE of the same
# command in separate --pmc passes (tools/collect_traffic.py keeps the classify kernel's dispatches, calibrated on the
# memory skeleton); D1 (reassembly): kernel stats.  F1's read bytes per packet (92.1) are bench.py flow_bytes for the
# owner-computed update (105.1 B per packet, 13 of them written: the 1-B compact list since round 6): the classify kernel no longer reads or writes the
# flows' counters, it writes an 8-B bucket entry instead (round 3's in-kernel atomics: 124.1).
set -o pipefail
T=${1:-r2}
O=gpurun_out/prof_$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
if [ ! -f $O/cal_fetch/cal_counter_collection.csv ]; then
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/cal_fetch -o cal -- tools/calib/stream_calib 1048576 4 > $O/cal_fetch.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/cal_write -o cal -- tools/calib/stream_calib 1048576 4 > $O/cal_write.log 2>&1 || exit 1
fi
B="bench.py --config F1 --steps 16 --warmup 4 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_F1 -o k -- python3 $B > $O/kt_F1.log 2>&1 || exit 1
python3 tools/f1_timed_stats.py $O/kt_F1/k_kernel_trace.csv --steps 16 --out $O/${T}_F1_timed.txt > /dev/null 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_F1 -o k -- python3 $B > $O/fetch_F1.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write_F1 -o k -- python3 $B > $O/write_F1.log 2>&1 || exit 1
python3 tools/collect_traffic.py --config F1 --fetch $O/fetch_F1/k_counter_collection.csv --write $O/write_F1/k_counter_collection.csv \
  --cal-fetch $O/cal_fetch/cal_counter_collection.csv --cal-write $O/cal_write/cal_counter_collection.csv \
  --n 1048576 --read-per-pkt 92.1 --write-per-pkt 13 --out $O/${T}_traffic_F1.json > $O/traffic_F1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_D1 -o k -- python3 bench.py --config D1 --no-cpu-baseline > $O/kt_D1.log 2>&1 || exit 1
# D1 traffic: 8 ppe_defrag calls alone (tools/defrag_run.py), every ppe_defrag kernel's FETCH / WRITE summed per call
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_D1 -o k -- python3 tools/defrag_run.py --calls 8 > $O/fetch_D1.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write_D1 -o k -- python3 tools/defrag_run.py --calls 8 > $O/write_D1.log 2>&1 || exit 1
AB=$(grep -o "alg_bytes_per_call [0-9.]*" $O/fetch_D1.log | awk '{print $2}')
python3 tools/collect_traffic.py --config D1 --kernel 'df_(?!init|age)' --calls 8 --alg-bytes $AB --n 65536 \
  --fetch $O/fetch_D1/k_counter_collection.csv --write $O/write_D1/k_counter_collection.csv \
  --cal-fetch $O/cal_fetch/cal_counter_collection.csv --cal-write $O/cal_write/cal_counter_collection.csv \
  --out $O/${T}_traffic_D1.json > $O/traffic_D1.log 2>&1 || exit 1
echo "stateful profiles done"
