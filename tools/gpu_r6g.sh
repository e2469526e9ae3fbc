# round 6: F1 owner update loading each bucket's first 16 B with its count (libppe_hip_f16) vs whole 64-B buckets
set -o pipefail
O=gpurun_out/r6g; mkdir -p $O
V=packet-process-engine_amd/libppe_hip_f16.so
PPE_LIB=$V timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flow.py tests/test_gpu_steer.py > $O/pytest_f16.txt 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --config F1 --no-cpu-baseline --steps 20 --warmup 5 > $O/base_$i.json 2> $O/base_$i.err || exit 1
  PPE_LIB=$V timeout -k 10 300 python bench.py --config F1 --no-cpu-baseline --steps 20 --warmup 5 > $O/f16_$i.json 2> $O/f16_$i.err || exit 1
done
echo rc=$?
