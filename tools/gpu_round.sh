set -o pipefail
mkdir -p gpurun_out/r2a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a/gputest.log 2>&1 && \
for c in C1 C2 C3 C4; do timeout -k 10 240 python -u bench.py --config $c --no-cpu-baseline --no-host-inclusive > gpurun_out/r2a/bench_$c.json 2> gpurun_out/r2a/bench_$c.err || exit 1; done
