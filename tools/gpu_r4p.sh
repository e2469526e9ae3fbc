# round 4: the flow table's 8-B global bucket path (tables past 2^23 slots) and the flow suite on the product build
set -o pipefail
O=gpurun_out/${1:-r4p}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_flow.py > $O/pytest_flow.txt 2>&1
