# round 4: D1 per-kernel instruction mix and waits (one SQ pass over 8 ppe_defrag calls)
set -o pipefail
O=gpurun_out/${1:-r4q}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES \
  --kernel-trace --output-format csv -d $O/sq_D1 -o k -- python3 tools/defrag_run.py --calls 8 > $O/sq_D1.log 2>&1
