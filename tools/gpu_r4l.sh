# round 4: where the owner-update kernel's time goes (diagnostic builds: 1 = gather only, 2 = neither phase)
set -o pipefail
O=gpurun_out/${1:-r4l}
mkdir -p $O
L=packet-process-engine_amd
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in ownerrec updab1 updab2; do  # (updab: wrong outputs, traces only)
  PPE_LIB=$L/libppe_hip_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o k -- \
    python3 bench.py --config F1 --steps 16 --warmup 4 --no-cpu-baseline > $O/kt_$v.log 2>&1 || exit 1
done
# the pre-launch event per batch vs host polling of the snapshot (PPE_FLOW_EVENT=0)
PPE_LIB=$L/libppe_hip_ownerrec.so PPE_FLOW_EVENT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_noev -o k -- \
  python3 bench.py --config F1 --steps 16 --warmup 4 --no-cpu-baseline > $O/kt_noev.log 2>&1 || exit 1
for i in 1 2; do
  PPE_LIB=$L/libppe_hip_ownerrec.so timeout -k 10 200 python bench.py --config F1 --no-cpu-baseline > $O/f1_ev_$i.json 2> $O/f1_ev_$i.err || exit 1
  PPE_LIB=$L/libppe_hip_ownerrec.so PPE_FLOW_EVENT=0 timeout -k 10 200 python bench.py --config F1 --no-cpu-baseline > $O/f1_noev_$i.json 2> $O/f1_noev_$i.err || exit 1
done
