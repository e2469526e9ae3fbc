set -o pipefail
O=gpurun_out/r4d; mkdir -p $O
L=packet-process-engine_amd; A="api=batches,bpl=0,outs=part"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_flow.py > $O/pytest.txt 2>&1 || exit 1
bash tools/gpu_ab_configs.sh r4d "C3" ph2=$L/libppe_hip.so:$A old=$L/libppe_hip_no2ph.so:$A -- --steps 20 --rounds 4 --check || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in old new old2 new2; do
  if [ ${v:0:3} = old ]; then export PPE_LIB=$L/libppe_hip_base.so; else unset PPE_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o k -- python3 bench.py --config F1 --steps 32 --warmup 8 --no-cpu-baseline > $O/$v.json 2> $O/$v.err || exit 1
done
