# new tests (flow table with a 4k-rule image; pipeline 5 variants), then A/B of the single-tile block walk
# (pipeline 5, 8 waves/SIMD) against the multi-tile kernel on C4 / C2 / C3
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
L=packet-process-engine_amd/libppe_hip.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flow.py \
  tests/test_gpu_parity.py -k "large_rule or every_kernel_variant or c3_64k or argument_errors" > $O/pytest.txt 2>&1 || exit 1
for c in C4 C2 C3; do
  timeout -k 10 300 python -u tools/ab_bench.py --config $c --steps 32 --rounds 4 --check \
    --variant mt=$L:api=batches,bpl=0 --variant sblk=$L:api=batches,bpl=0,pipeline=5 > $O/ab_$c.txt 2>&1 || exit 1
done
