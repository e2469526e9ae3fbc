set -o pipefail
O=gpurun_out/r6b; mkdir -p $O
bash tools/gpu_bench_ab.sh r6b F1 packet-process-engine_amd/libppe_hip_base.so tests/test_gpu_defrag.py && \
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
echo rc=$?
