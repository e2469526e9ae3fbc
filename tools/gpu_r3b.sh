# round 3: GPU suite, smoke, default bench line, then the same stateless configs with compact leaves off (A/B)
set -o pipefail
O=gpurun_out/${1:-r3b}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err && \
PPE_COMPACT=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive > $O/bench_nocompact.json 2> $O/bench_nocompact.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive > $O/bench2.json 2> $O/bench2.err
