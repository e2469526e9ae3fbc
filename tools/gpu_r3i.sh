# Round 3: flow-table slot record (last-seen beside the packed counters) — flow GPU tests, then F1 with the previous
# layout (libppe_hip_base.so) and the new one, alternating, each a bench.py process of its own
set -o pipefail
O=gpurun_out/r3i; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_flow.py tests/test_gpu_steer.py > $O/pytest_flow.txt 2>&1 || exit 1
for i in 1 2; do
  PPE_LIB=packet-process-engine_amd/libppe_hip_base.so timeout -k 10 300 python bench.py --config F1 --steps 32 --warmup 8 --no-cpu-baseline > $O/f1_base_$i.json 2> $O/f1_base_$i.err || exit 1
  timeout -k 10 300 python bench.py --config F1 --steps 32 --warmup 8 --no-cpu-baseline > $O/f1_new_$i.json 2> $O/f1_new_$i.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 120 rocprofv3 -L > $O/counters_avail.txt 2>&1 || true
