# round 4: D1 per-kernel traffic (FETCH_SIZE / WRITE_SIZE passes of 8 ppe_defrag calls) and durations
set -o pipefail
O=gpurun_out/${1:-r4n}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt_D1 -o k -- python3 tools/defrag_run.py --calls 8 > $O/kt_D1.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_D1 -o k -- python3 tools/defrag_run.py --calls 8 > $O/fetch_D1.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write_D1 -o k -- python3 tools/defrag_run.py --calls 8 > $O/write_D1.log 2>&1 || exit 1
python3 tools/kernel_traffic.py --fetch $O/fetch_D1/k_counter_collection.csv --write $O/write_D1/k_counter_collection.csv \
  --trace $O/kt_D1/k_kernel_trace.csv --calls 8 > $O/traffic_D1.txt 2>&1
