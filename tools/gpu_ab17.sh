# D1: the assembly with every load of a segment issued first (passes of 64 U output dwords, U = 2 / 4 / 8) vs the
# previous assembly, interleaved bench runs
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
D=packet-process-engine_amd
for r in 1 2; do
  for v in olddf dfu2 dfu4 dfu8; do
    PPE_LIB=$D/libppe_hip_$v.so timeout -k 10 300 python -u bench.py --config D1 --no-cpu-baseline > $O/$v.$r.json 2> $O/$v.$r.err || exit 1
  done
done
