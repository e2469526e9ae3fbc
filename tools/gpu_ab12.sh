# F1 A/B: conditional last-seen store (PPE_LAST_COND) vs the per-packet store, interleaved bench runs on one box
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
D=packet-process-engine_amd
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --config F1 --no-cpu-baseline > $O/base$r.json 2> $O/base$r.err || exit 1
  PPE_LIB=$D/libppe_hip_lastc.so timeout -k 10 200 python -u bench.py --config F1 --no-cpu-baseline > $O/lastc$r.json 2> $O/lastc$r.err || exit 1
done
