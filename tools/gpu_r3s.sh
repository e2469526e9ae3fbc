# Round-3 evidence with the current kernels: rehearsal (GPU suite, smoke, default bench), then the profile set
set -o pipefail
bash tools/gpu_final.sh r3s && \
timeout -k 10 1200 bash tools/profile_round.sh r3s "C1 C2 C3 C4" > gpurun_out/r3s/profile_round.log 2>&1 && \
timeout -k 10 900 bash tools/profile_stateful.sh r3s > gpurun_out/r3s/profile_stateful.log 2>&1
