# round 4 evidence with the product kernels on one box: the rehearsal (GPU suite, smoke, default bench line), then the
# profile sets of the stateless configs and of the stateful rows:  bash tools/gpu_r4final.sh TAG
set -o pipefail
T=$1
bash tools/gpu_final.sh $T && \
timeout -k 10 600 bash tools/profile_round.sh $T "C1 C2 C3 C4" > gpurun_out/$T/profile_round.log 2>&1 && \
timeout -k 10 300 bash tools/profile_stateful.sh $T > gpurun_out/$T/profile_stateful.log 2>&1
