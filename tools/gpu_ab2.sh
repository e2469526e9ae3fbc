set -o pipefail
O=gpurun_out/r2n
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=packet-process-engine_amd
for v in "" _abl1 _abl2 _abl4 _abl8 _abl15; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SMEM --kernel-trace --output-format csv -d $O/pmc$v -o c1 -- python3 tools/ring_run.py --config C1 --batches 32 --launches 2 --lib $P/libppe_hip$v.so > $O/pmc$v.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $O/pmc$v/c1_counter_collection.csv --tiles $((32 * 16384)) --min-us 100 > $O/sq$v.txt 2>&1
done
