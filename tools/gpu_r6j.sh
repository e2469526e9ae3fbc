# round 6: LLVM AMDGPU machine-scheduler strategies for the classify kernels (max-ilp / max-memory-clause /
# iterative-ilp builds of csrc/ppe_kernels.hip) against the product build, C1..C4 in-process A/B
set -o pipefail
O=gpurun_out/r6j; mkdir -p $O
L=packet-process-engine_amd
for C in C1 C4 C3 C2; do
  timeout -k 10 300 python -u tools/ab_bench.py --config $C --rounds 5 --steps 32 --check \
    --variant base=$L/libppe_hip.so --variant ilp=$L/libppe_hip_maxilp.so --variant mem=$L/libppe_hip_maxmemoryclause.so \
    --variant iter=$L/libppe_hip_iterativeilp.so > $O/ab_$C.txt 2>&1 || exit 1
done
echo rc=$?
