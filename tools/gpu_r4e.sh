# round 4: F1 flow pipeline variants (libppe_hip_owner.so: claims inside the classify launch, finalize finds the
# slots; PPE_FLOW_OWNER=1 adds the owner-computed FlowUpdate): flow + steer tests on both, then F1 A/B vs product
set -o pipefail
O=gpurun_out/${1:-r4e}
mkdir -p $O
L=packet-process-engine_amd
NEW=$L/libppe_hip_owner.so
PPE_LIB=$NEW PPE_FLOW_OWNER=0 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_flow.py > $O/pytest_flow_claim.txt 2>&1 || exit 1
PPE_LIB=$NEW timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_flow.py \
  tests/test_gpu_steer.py > $O/pytest_flow_owner.txt 2>&1 || exit 1
for i in 1 2; do
  PPE_LIB=$L/libppe_hip.so timeout -k 10 200 python bench.py --config F1 --no-cpu-baseline > $O/f1_base_$i.json 2> $O/f1_base_$i.err || exit 1
  PPE_LIB=$NEW PPE_FLOW_OWNER=0 timeout -k 10 200 python bench.py --config F1 --no-cpu-baseline > $O/f1_claim_$i.json 2> $O/f1_claim_$i.err || exit 1
  PPE_LIB=$NEW timeout -k 10 200 python bench.py --config F1 --no-cpu-baseline > $O/f1_owner_$i.json 2> $O/f1_owner_$i.err || exit 1
done
