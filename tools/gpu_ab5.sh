set -o pipefail
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "flow or steer" > $O/pytest.txt 2>&1 || exit 1
for r in 1 2; do
timeout -k 10 300 python -u bench.py --config F1 --no-cpu-baseline > $O/f1_$r.json 2> $O/f1_$r.err || exit 1
done
