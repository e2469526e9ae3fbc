# direct-record leaves: C3 parity (default image, pipeline 5, kernel variants), then C3 with the leaf cap (default for
# >= 16k rules) against the uncapped image (PPE_LEAF_CAP_DEPTH=0), one process each, alternating
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
L=packet-process-engine_amd/libppe_hip.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "c3_64k or every_kernel_variant or golden or config_batches" > $O/pytest.txt 2>&1 || exit 1
run() {
  env $2 timeout -k 10 300 python -u tools/ab_bench.py --config C3 --steps 32 --rounds 3 \
    --variant cur=$L:api=batches,bpl=0 > $O/ab_$1.txt 2>&1 || exit 1
  grep "kernel med" $O/ab_$1.txt | sed "s/^/$1 /" >> $O/summary.txt
}
run off1 PPE_LEAF_CAP_DEPTH=0 && run drec1 X=1 && run d10 PPE_LEAF_CAP_DEPTH=10 && run off2 PPE_LEAF_CAP_DEPTH=0 && run drec2 X=1
