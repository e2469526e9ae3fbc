# Round 3: (1) branchless LDS block walk A/B on C4 / C2 against the product (2-tile pipelined loop) and the round-2
# loop; (2) memory-pipeline counters (TA / TD / TCP latency, VMEM level, LDS conflicts) for C1, C4 and C3
set -o pipefail
L=packet-process-engine_amd
O="api=batches,bpl=0,outs=part"
for C in C4 C2; do
  bash tools/gpu_ab.sh r3j $C prod=$L/libppe_hip.so:$O bl=$L/libppe_hip_bl.so:$O r2loop=$L/libppe_hip_r2loop.so:$O \
    -- --steps 20 --rounds 4 --check || exit 1
done
D=gpurun_out/r3j; K=32
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
P1="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P3="TCP_TCP_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT"
for C in C1 C4 C3; do
  R="tools/ring_run.py --config $C --batches $K --launches 3"
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $D/p${i}_$C -o k -- python3 $R > $D/p${i}_$C.log 2>&1 || exit 1
    python3 tools/pmc_summary.py $D/p${i}_$C/k_counter_collection.csv --tiles $((K * 16384)) --min-us 50 >> $D/pmc_$C.txt 2>&1
  done
done
