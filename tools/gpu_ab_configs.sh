# Interleaved in-process A/B of several libraries / settings over several configs on one GPU box:
#   tools/gpu_ab_configs.sh TAG "C4 C3 C2" VARIANT... [-- extra ab_bench.py args]
# VARIANT = name=libpath[:key=val,...] as tools/ab_bench.py takes it (E_NAME=value sets an environment variable for
# that variant).  Each config runs through tools/gpu_ab.sh; the "kernel med" lines collect in gpurun_out/TAG/summary.txt.
# Round-3 runs recorded in profiles/r3_ab_runs.md used it as, e.g. (L=packet-process-engine_amd, O=api=batches,bpl=0,outs=part):
#   r5   C3 "cut=$L/libppe_hip.so:$O multi=$L/libppe_hip.so:pipeline=3,$O"           (cut lists vs block walk)
#   r3g  "C4 C3" "full=$L/libppe_hip.so none=$L/libppe_hip_abl15.so ..."             (ablation builds)
#   r3h / r3j / r3k / r3p  "C4 C3 C2" "new=$L/libppe_hip.so:$O old=$L/libppe_hip_bl.so:$O" -- --steps 20 --rounds 4 --check
set -o pipefail
T=$1; CFGS=$2; shift 2
for C in $CFGS; do
  bash tools/gpu_ab.sh $T $C "$@" || exit 1
done
