set -o pipefail
O=gpurun_out/$1
mkdir -p $O
P=packet-process-engine_amd
shift
timeout -k 10 400 python -u tools/ab_bench.py --nbufs 8 --steps 32 --rounds 5 --check "$@" > $O/ab.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1
