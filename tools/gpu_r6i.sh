# round 6: F1 / D1 with warm-ups that keep the config's state in the Infinity Cache (bench.py), F1 timed region traced
set -o pipefail
O=gpurun_out/r6i; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py --config F1 --no-cpu-baseline --steps 20 --warmup 5 > $O/F1_$i.json 2> $O/F1_$i.err || exit 1
done
timeout -k 10 300 python bench.py --config D1 --no-cpu-baseline --steps 20 --warmup 5 > $O/D1.json 2> $O/D1.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_F1 -o k -- python3 bench.py --config F1 --steps 16 --warmup 4 --no-cpu-baseline > $O/kt_F1.log 2>&1 || exit 1
python3 tools/f1_timed_stats.py $O/kt_F1/k_kernel_trace.csv --steps 16 --out $O/F1_timed.txt
echo rc=$?
