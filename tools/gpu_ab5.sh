set -o pipefail
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || exit 1
for r in 1 2; do
PPE_FLOW_FOLD_SWEEP=-1 timeout -k 10 300 python -u bench.py --config F1 --configs= --no-cpu-baseline --no-host-inclusive > $O/f1_inline_$r.json 2> $O/f1_inline_$r.err || exit 1
timeout -k 10 300 python -u bench.py --config F1 --configs= --no-cpu-baseline --no-host-inclusive > $O/f1_sched_$r.json 2> $O/f1_sched_$r.err || exit 1
done
