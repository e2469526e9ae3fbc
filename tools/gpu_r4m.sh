# round 4: finalize and the owner update in one post-classify launch (libppe_hip_post.so) vs two launches
# (libppe_hip_ownerrec.so), both with the host polling the snapshot instead of a per-batch event
set -o pipefail
O=gpurun_out/${1:-r4m}
mkdir -p $O
L=packet-process-engine_amd
export PPE_FLOW_EVENT=0
PPE_LIB=$L/libppe_hip_post.so timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_flow.py tests/test_gpu_steer.py > $O/pytest_flow_post.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
PPE_LIB=$L/libppe_hip_post.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_post -o k -- \
  python3 bench.py --config F1 --steps 16 --warmup 4 --no-cpu-baseline > $O/kt_post.log 2>&1 || exit 1
for i in 1 2; do
  for v in post ownerrec; do
    PPE_LIB=$L/libppe_hip_$v.so timeout -k 10 200 python bench.py --config F1 --no-cpu-baseline > $O/f1_${v}_$i.json 2> $O/f1_${v}_$i.err || exit 1
  done
done
