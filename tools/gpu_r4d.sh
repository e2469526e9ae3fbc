# round 4: where the C3 multi-tile round spends its time (phase stamps), then the round-end rehearsal
set -o pipefail
O=gpurun_out/${1:-r4d}
mkdir -p $O
L=packet-process-engine_amd
timeout -k 10 200 python -u tools/trace_mt.py --lib $L/libppe_hip_mttrace.so --config C3 > $O/trace_mt_C3.txt 2>&1 && \
bash tools/gpu_final.sh ${1:-r4d}
rc=$?
# (rc 1: a failed test or bench line, no fault: the A/B still runs)
[ $rc -le 1 ] && timeout -k 10 240 python -u tools/ab_defrag.py --variant base=$L/libppe_hip.so --variant asm1=$L/libppe_hip_asm1.so \
  --variant asm2=$L/libppe_hip_asm2.so --variant asm4=$L/libppe_hip_asm4.so > $O/ab_defrag.txt 2>&1
# F1: what the per-packet counter atomic (16) and the last-seen store (32) cost today
for v in abl16 abl32 abl48 base; do
  lib=$L/libppe_hip_$v.so; [ $v = base ] && lib=$L/libppe_hip.so
  PPE_LIB=$lib timeout -k 10 200 python bench.py --config F1 --no-cpu-baseline > $O/f1_$v.json 2> $O/f1_$v.err || break
done
