# round 4: D1 process kernel without the fragment ids (the stash keeps a held fragment's id, the place kernel reads
# this batch's from the input) and with 4-word records in its window (noid: 16 deep, noid8: 8 deep)
set -o pipefail
O=gpurun_out/${1:-r4aa}
mkdir -p $O
L=packet-process-engine_amd
PPE_LIB=$L/libppe_hip_dfnoid.so timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_defrag.py tests/test_gpu_mbuf.py > $O/pytest_defrag.txt 2>&1 || exit 1
PPE_LIB=$L/libppe_hip_dfnoid8.so timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_gpu_defrag.py > $O/pytest_defrag8.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_defrag.py --variant head=$L/libppe_hip_dfhead.so --variant noid=$L/libppe_hip_dfnoid.so \
  --variant noid8=$L/libppe_hip_dfnoid8.so > $O/ab_defrag.txt 2>&1
