set -o pipefail
O=gpurun_out/r2i
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R="tools/ring_run.py --config C1 --batches 32 --launches 3"
timeout -k 10 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/a -o c1 -- python3 $R > $O/a.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC --kernel-trace --output-format csv -d $O/b -o c1 -- python3 $R > $O/b.log 2>&1
python3 tools/pmc_summary.py $O/a/c1_counter_collection.csv $O/b/c1_counter_collection.csv --tiles $((32 * 16384)) --min-us 100 > $O/sq_summary.txt 2>&1
