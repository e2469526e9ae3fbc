# memory-pipeline counters of the multi-tile (C3) and single-tile (C1) classify kernels over tools/ring_run.py
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1
for C in C3 C1; do
  R="tools/ring_run.py --config $C --batches 32 --launches 3"
  timeout -s KILL 150 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/ta_$C -o k -- python3 $R > $O/ta_$C.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $O/ta_$C/k_counter_collection.csv --tiles $((32 * 16384)) --min-us 50 > $O/ta_$C.txt 2>&1
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $O/sq_$C -o k -- python3 $R > $O/sq_$C.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $O/sq_$C/k_counter_collection.csv --tiles $((32 * 16384)) --min-us 50 > $O/sq_$C.txt 2>&1
  timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-trace --output-format csv -d $O/tcc_$C -o k -- python3 $R > $O/tcc_$C.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $O/tcc_$C/k_counter_collection.csv --tiles $((32 * 16384)) --min-us 50 > $O/tcc_$C.txt 2>&1
done
