# round 4: D1 assembly with n / S waves striding over the slots (empty slots S per wave, datagrams one per wave)
# (procpf: stride 4 + the process loop waiting one round trip per fragment)
set -o pipefail
O=gpurun_out/${1:-r4o}
mkdir -p $O
L=packet-process-engine_amd
for v in asms2 asms4 procpf; do
  PPE_LIB=$L/libppe_hip_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_defrag.py > $O/pytest_defrag_$v.txt 2>&1 || exit 1
done
timeout -k 10 240 python -u tools/ab_defrag.py --variant base=$L/libppe_hip.so --variant s2=$L/libppe_hip_asms2.so \
  --variant s4=$L/libppe_hip_asms4.so --variant s4pf=$L/libppe_hip_procpf.so > $O/ab_defrag.txt 2>&1
