# C3 / C4: leaf threshold binth 1 (default) against 2 and 3 on the multi-tile block walk (separate processes: the
# image is built at commit from PPE_BINTH)
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
L=packet-process-engine_amd/libppe_hip.so
for c in C3 C4; do
  for b in 1 2 3 1; do
    timeout -k 10 300 python -u tools/ab_bench.py --config $c --steps 32 --rounds 3 --binth $b \
      --variant cur=$L:api=batches,bpl=0 > $O/ab_${c}_b$b.txt 2>&1 || exit 1
  done
done
