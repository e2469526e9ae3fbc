# round 4: the defrag GPU tests with the 524,288-fragment look-back batch (product build)
set -o pipefail
O=gpurun_out/${1:-r4z}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_defrag.py \
  > $O/pytest_defrag.txt 2>&1
