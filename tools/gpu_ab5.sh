set -o pipefail
O=gpurun_out/$1
mkdir -p $O
P=packet-process-engine_amd
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || exit 1
for C in C1 C1; do
timeout -k 10 400 python -u tools/ab_bench.py --config $C --steps 32 --rounds 3 --check \
  --variant blocks=$P/libppe_hip.so:api=batches,bpl=0 --variant nodes=$P/libppe_hip_stnode.so:api=batches,bpl=0 >> $O/ab_$C.txt 2>&1 || exit 1
done
