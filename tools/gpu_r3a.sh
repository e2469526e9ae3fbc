set -o pipefail
O=gpurun_out/r3a
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 20 --warmup 5 --configs C4 --no-cpu-baseline --no-host-inclusive > $O/bench_kt.json 2> $O/bench_kt.err
