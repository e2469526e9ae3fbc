# Round 3: defrag without its scan launches (13 launches per call instead of 17) — defrag GPU tests, then D1 with
# the previous library (libppe_hip_bl.so) and the new one, alternating processes
set -o pipefail
O=gpurun_out/r3q; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_defrag.py > $O/pytest_defrag.txt 2>&1 || exit 1
for i in 1 2; do
  PPE_LIB=packet-process-engine_amd/libppe_hip_bl.so timeout -k 10 300 python bench.py --config D1 --no-cpu-baseline > $O/d1_old_$i.json 2> $O/d1_old_$i.err || exit 1
  timeout -k 10 300 python bench.py --config D1 --no-cpu-baseline > $O/d1_new_$i.json 2> $O/d1_new_$i.err || exit 1
done
