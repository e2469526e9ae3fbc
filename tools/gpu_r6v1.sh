# round 6 evidence (r6h, then r6v after the completion words and F1 region change), part 1: the round-end rehearsal (GPU suite, smoke, the driver's bench command) and the stateful
# profiles (F1 timed region, D1)
set -o pipefail
T=${1:-r6v}
bash tools/gpu_final.sh $T && \
timeout -k 10 900 bash tools/profile_stateful.sh $T > gpurun_out/$T/profile_stateful.log 2>&1
echo rc=$?
