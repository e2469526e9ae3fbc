set -o pipefail
O=gpurun_out/${1:-r2o}
mkdir -p $O
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && \
timeout -k 10 400 python -u bench.py --configs "" --no-cpu-baseline --no-host-inclusive > $O/bench2.json 2> $O/bench2.err && \
timeout -k 10 400 python -u bench.py --configs "" --no-cpu-baseline --no-host-inclusive --steps 20 --warmup 5 > $O/bench3.json 2> $O/bench3.err
