# round 6: GPU suite after trimming unreachable kernel instantiations; the cut-list kernel over a whole-LDS image
# compiled for 7 waves per SIMD (PPE_CUT_LDS_WAVES=7: 94 SGPRs, 12 spilled to VGPR lanes instead of 28 at 78; still 8
# waves resident) against the product, C4 / C2 in-process A/B
set -o pipefail
O=gpurun_out/r6ab; mkdir -p $O
L=packet-process-engine_amd
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest.txt 2>&1 || exit 1
for C in C4 C2; do
  timeout -k 10 300 python -u tools/ab_bench.py --config $C --rounds 7 --steps 32 --check \
    --variant base=$L/libppe_hip.so --variant cw7=$L/libppe_hip_cw7.so > $O/ab_$C.txt 2>&1 || exit 1
done
grep -h "kernel med\|identical\|differ" $O/ab_C*.txt
tail -1 $O/pytest.txt
