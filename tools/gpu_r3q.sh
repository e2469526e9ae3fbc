# Round 3: defrag A/B (R3Q = output tag) — defrag GPU tests, then D1 with libppe_hip_bl.so (old) and the product (new),
# alternating processes
set -o pipefail
O=gpurun_out/${R3Q:-r3q}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_defrag.py > $O/pytest_defrag.txt 2>&1 || exit 1
for i in 1 2; do
  PPE_LIB=packet-process-engine_amd/${OLD_LIB:-libppe_hip_bl.so} timeout -k 10 300 python bench.py --config D1 --no-cpu-baseline > $O/d1_old_$i.json 2> $O/d1_old_$i.err || exit 1
  timeout -k 10 300 python bench.py --config D1 --no-cpu-baseline > $O/d1_new_$i.json 2> $O/d1_new_$i.err || exit 1
done
