set -o pipefail
O=gpurun_out/$1
mkdir -p $O
P=packet-process-engine_amd
for C in C2 C4 C3; do
timeout -k 10 400 python -u tools/ab_bench.py --config $C --nbufs 8 --steps 32 --rounds 3 --check \
  --variant new=$P/libppe_hip.so:api=batches,bpl=0 --variant prev=$P/libppe_hip_prev.so:api=batches,bpl=0 > $O/ab_$C.txt 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1
