# round 6: the cut-list kernel over a whole-LDS image compiled for 7 waves per SIMD (PPE_CUT_LDS_WAVES=7, fewer SGPR
# spills) against the product, in the bench's layout (part8 compact lists), with the grid the occupancy query gives
# and with 1 / 2 workgroups per CU forced (the query reports 1 for the 7-wave build): C4, C2
set -o pipefail
O=gpurun_out/r6ac; mkdir -p $O
L=packet-process-engine_amd
export TMPDIR=/tmp
for C in C4 C2; do
  timeout -k 10 300 python -u tools/ab_bench.py --config $C --rounds 7 --steps 32 --check \
    --variant base=$L/libppe_hip.so:outs=part8 --variant cw7=$L/libppe_hip_cw7.so:outs=part8 \
    --variant base1=$L/libppe_hip.so:outs=part8,blocks_per_cu=1 --variant cw7x2=$L/libppe_hip_cw7.so:outs=part8,blocks_per_cu=2 \
    > $O/ab_$C.txt 2>&1 || exit 1
done
grep -h "kernel med\|identical\|differ" $O/ab_C*.txt
