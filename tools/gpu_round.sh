set -o pipefail
O=gpurun_out/${1:-r2j}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 && \
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 300 python -u bench.py --scaling strong --configs C4 --no-cpu-baseline --no-host-inclusive > $O/bench_strong.json 2> $O/bench_strong.err
