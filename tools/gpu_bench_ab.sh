# A/B of the product library against another build on one bench config, alternating processes (the stateful configs,
# whose calls are not ring launches that tools/ab_bench.py interleaves):
#   tools/gpu_bench_ab.sh TAG CONFIG OLD_LIB [PYTEST_FILE] [-- extra bench.py args]
# Runs PYTEST_FILE's GPU tests first (if given), then 2 x (old, new) bench.py --config CONFIG lines into
# gpurun_out/TAG/{old,new}_N.json.  Round 3 used it for F1 (r3i: tests/test_gpu_flow.py) and D1 (r3q..r3u:
# tests/test_gpu_defrag.py) against libppe_hip_base.so / libppe_hip_bl.so.
set -o pipefail
T=$1; C=$2; OLD=$3; shift 3
TF=""; [ $# -gt 0 ] && [ "$1" != "--" ] && { TF=$1; shift; }
[ "$1" = "--" ] && shift
O=gpurun_out/$T; mkdir -p $O
if [ -n "$TF" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread $TF > $O/pytest.txt 2>&1 || exit 1
fi
for i in 1 2; do
  PPE_LIB=$OLD timeout -k 10 300 python bench.py --config $C --no-cpu-baseline "$@" > $O/old_$i.json 2> $O/old_$i.err || exit 1
  timeout -k 10 300 python bench.py --config $C --no-cpu-baseline "$@" > $O/new_$i.json 2> $O/new_$i.err || exit 1
done
