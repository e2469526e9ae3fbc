# round 6: C1's kernel variant built under the iterative-ILP scheduler in its own translation unit
# (csrc/ppe_kernels_hoist.hip), the others unchanged: GPU suite, in-process A/B against the previous build
# (libppe_hip_base.so) on C1 (9 rounds) and C2 (5), then default bench lines alternating
set -o pipefail
O=gpurun_out/r6t; mkdir -p $O
L=packet-process-engine_amd
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_bench.py --config C1 --rounds 9 --steps 32 --check \
  --variant base=$L/libppe_hip_base.so --variant new=$L/libppe_hip.so > $O/ab_C1.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_bench.py --config C2 --rounds 5 --steps 32 --check \
  --variant base=$L/libppe_hip_base.so --variant new=$L/libppe_hip.so > $O/ab_C2.txt 2>&1 || exit 1
for i in 1 2; do
  for V in base new; do
    LIB=$L/libppe_hip_$V.so; [ $V = new ] && LIB=$L/libppe_hip.so
    PPE_LIB=$LIB timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/all_${V}_$i.json 2> $O/all_${V}_$i.err || exit 1
  done
done
grep -h "kernel med\|identical\|differ" $O/ab_C*.txt
for f in $O/all_*_[12].json; do echo $f $(python -c "
import json,sys; d=json.load(open(sys.argv[1])); c=d.get('configs',{})
print(d['value'], d['ms_per_step'], d['roofline']['us_per_1M_packets'], {k: round(v.get('ms_per_step',0)*1e3,2) for k,v in c.items()})" $f); done
tail -1 $O/pytest.txt
