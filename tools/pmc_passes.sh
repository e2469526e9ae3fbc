#!/bin/bash
# Extra PMC passes over the C1 bench (issue / LDS / clock evidence), one rocprofv3 run per counter group.
#   usage (GPU box, repo root): bash tools/pmc_passes.sh TAG   → gpurun_out/pmc_TAG/...
set -e
T=${1:-x}
O=gpurun_out/pmc_$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P="bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-host-inclusive"
rocprofv3 -L > $O/counters_list.txt 2>&1 || true
i=0
for G in "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $O/p$i -o c1 -- python3 $P > $O/p$i.log 2>&1 || echo "pass $i failed"
  python3 tools/pmc_summary.py $O/p$i/c1_counter_collection.csv >> $O/summary.txt 2>&1 || true
done
echo pmc done
