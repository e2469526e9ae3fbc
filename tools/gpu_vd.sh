set -o pipefail
O=gpurun_out/$1; mkdir -p $O
P=packet-process-engine_amd
for c in C1 C4 C2; do
echo "== outsfixed $c" >> $O/diff.txt
timeout -k 10 200 python -u tools/variant_diff.py $P/libppe_hip_outsfixed.so --part --config $c >> $O/diff.txt 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || exit 1
for C in C1 C4 C1; do
timeout -k 10 400 python -u tools/ab_bench.py --config $C --steps 32 --rounds 3 --check \
  --variant cur=$P/libppe_hip.so:api=batches,bpl=0,outs=part --variant fixed=$P/libppe_hip_outsfixed.so:api=batches,bpl=0,outs=part >> $O/ab.txt 2>&1 || exit 1
done
