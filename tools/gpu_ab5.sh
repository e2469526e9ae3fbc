set -o pipefail
O=gpurun_out/$1
mkdir -p $O
P=packet-process-engine_amd
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-host-inclusive > $O/bench_part.json 2> $O/bench_part.err || exit 1
PPE_NO_PART=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-host-inclusive > $O/bench_nopart.json 2> $O/bench_nopart.err || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-host-inclusive --configs= > $O/bench_part2.json 2> $O/bench_part2.err || exit 1
