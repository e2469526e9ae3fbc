# round 6: classify launches tracked by a completion word their last workgroup writes to pinned memory instead of an
# event marker behind every launch (image / ring readers).  The whole GPU suite on the product, then bench lines
# against the previous build (libppe_hip_base.so), alternating processes, and an F1 kernel trace
set -o pipefail
O=gpurun_out/r6r; mkdir -p $O
L=packet-process-engine_amd
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest.txt 2>&1 || exit 1
for i in 1 2 3; do
  for V in base new; do
    LIB=$L/libppe_hip_$V.so; [ $V = new ] && LIB=$L/libppe_hip.so
    PPE_LIB=$LIB timeout -k 10 300 python bench.py --config F1 --steps 20 --warmup 5 --no-cpu-baseline > $O/F1_${V}_$i.json 2> $O/F1_${V}_$i.err || exit 1
  done
done
for i in 1 2; do
  for V in base new; do
    LIB=$L/libppe_hip_$V.so; [ $V = new ] && LIB=$L/libppe_hip.so
    PPE_LIB=$LIB timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/all_${V}_$i.json 2> $O/all_${V}_$i.err || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_new -o run --output-format csv -- python bench.py --config F1 --steps 16 --warmup 5 --no-cpu-baseline > $O/prof_new.log 2>&1 || exit 1
for f in $O/F1_*_[123].json; do echo $f $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" $f); done
for f in $O/all_*_[12].json; do echo $f $(python -c "
import json,sys; d=json.load(open(sys.argv[1])); c=d.get('configs',{})
print(d['value'], d['ms_per_step'], {k: round(v.get('ms_per_step',0)*1e3,2) for k,v in c.items()})" $f); done
python tools/f1_timed_stats.py $O/prof_new/run_kernel_trace.csv --steps 16
tail -1 $O/pytest.txt
