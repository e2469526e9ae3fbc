# round 6 evidence (r6h, then r6v), part 2: the stateless configs' kernel traces, calibrated traffic, TCC and SQ counters
set -o pipefail
T=${1:-r6v}
mkdir -p gpurun_out/$T
timeout -k 10 1100 bash tools/profile_round.sh $T "C1 C2 C3 C4" > gpurun_out/$T/profile_round.log 2>&1
echo rc=$?
