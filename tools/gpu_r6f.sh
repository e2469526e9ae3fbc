# round 6: cut-lookup candidates per round from LDS (PPE_CUT_W_LDS 1 / 2 (base) / 3 / 4), C4 and C2
set -o pipefail
O=gpurun_out/r6f; mkdir -p $O
L=packet-process-engine_amd
for C in C4 C2; do
  timeout -k 10 300 python -u tools/ab_bench.py --config $C --rounds 7 --steps 32 --check \
    --variant base=$L/libppe_hip.so --variant w1=$L/libppe_hip_w1.so --variant w3=$L/libppe_hip_w3.so \
    --variant w4=$L/libppe_hip_w4.so > $O/ab_$C.txt 2>&1 || exit 1
done
echo rc=$?
