# Dynamic instruction mix per tile of library variants (one rocprofv3 --pmc pass each over tools/ring_run.py):
#   bash tools/gpu_sq_variants.sh TAG "C4 C3" name=lib.so ...     → gpurun_out/TAG/sq_<config>_<name>.txt
set -o pipefail
T=$1; CONFIGS=$2; shift 2
D=gpurun_out/$T; mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
K=32
P="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY"
for C in $CONFIGS; do
  for V in "$@"; do
    N=${V%%=*}; LIB=${V#*=}
    timeout -s KILL 150 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $D/sq_${C}_$N -o k -- python3 tools/ring_run.py --config $C --batches $K --launches 3 --lib $LIB > $D/sq_${C}_$N.log 2>&1 || exit 1
    python3 tools/pmc_summary.py $D/sq_${C}_$N/k_counter_collection.csv --tiles $((K * 16384)) --min-us 50 > $D/sq_${C}_$N.txt 2>&1
  done
done
