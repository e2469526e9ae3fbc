# round 4: owner-update buckets staged in LDS (4-B entries, one 64-B segment per bucket; libppe_hip_ownerlds.so) vs
# 8-B global entries (libppe_hip_ownerg.so): flow tests on both, kernel trace, F1 A/B vs product
set -o pipefail
O=gpurun_out/${1:-r4i}
mkdir -p $O
L=packet-process-engine_amd
for v in ownerlds ownerg; do
  PPE_LIB=$L/libppe_hip_$v.so timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_flow.py tests/test_gpu_steer.py > $O/pytest_flow_$v.txt 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in ownerlds ownerg; do
  PPE_LIB=$L/libppe_hip_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o k -- \
    python3 bench.py --config F1 --steps 16 --warmup 4 --no-cpu-baseline > $O/kt_$v.log 2>&1 || exit 1
done
for i in 1 2; do
  for v in ownerlds ownerg; do
    PPE_LIB=$L/libppe_hip_$v.so timeout -k 10 200 python bench.py --config F1 --no-cpu-baseline > $O/f1_${v}_$i.json 2> $O/f1_${v}_$i.err || exit 1
  done
  PPE_LIB=$L/libppe_hip.so timeout -k 10 200 python bench.py --config F1 --no-cpu-baseline > $O/f1_base_$i.json 2> $O/f1_base_$i.err || exit 1
done
