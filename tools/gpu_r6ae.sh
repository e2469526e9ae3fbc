# round 6: the cut-list entry test with each prefix check as ~(m ^ (m - 1)) (one add and one 3-input bit operation
# per address, one compare for both) against the previous build (libppe_hip_base.so): the GPU parity tests, then
# C4 / C2 / C3 in-process A/B in the bench layout
set -o pipefail
O=gpurun_out/r6ae; mkdir -p $O
L=packet-process-engine_amd
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_packed.py > $O/pytest.txt 2>&1 || exit 1
for C in C4 C2 C3; do
  timeout -k 10 300 python -u tools/ab_bench.py --config $C --rounds 7 --steps 32 --check \
    --variant base=$L/libppe_hip_base.so:outs=part8 --variant new=$L/libppe_hip.so:outs=part8 > $O/ab_$C.txt 2>&1 || exit 1
done
grep -h "kernel med\|identical\|differ" $O/ab_C*.txt
tail -1 $O/pytest.txt
