# round 6: flow tests on the dense-run update build, F1 A/B (dense vs base), the driver's bench command
set -o pipefail
O=gpurun_out/r6e; mkdir -p $O
PPE_LIB=packet-process-engine_amd/libppe_hip_dense.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flow.py tests/test_gpu_steer.py > $O/pytest_dense.txt 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py --config F1 --no-cpu-baseline --steps 20 --warmup 5 > $O/base_$i.json 2> $O/base_$i.err || exit 1
  PPE_LIB=packet-process-engine_amd/libppe_hip_dense.so timeout -k 10 300 python bench.py --config F1 --no-cpu-baseline --steps 20 --warmup 5 > $O/dense_$i.json 2> $O/dense_$i.err || exit 1
done
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo rc=$?
