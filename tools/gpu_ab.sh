# One interleaved in-process A/B run on the GPU box (replaces round 2's one-off gpu_abN.sh scripts):
#   tools/gpu_ab.sh OUTDIR CONFIG VARIANT... [-- extra ab_bench.py args]
# VARIANT = name=libpath[:key=val,...] as tools/ab_bench.py takes it (E_NAME=value sets an environment variable for
# that variant, e.g. E_PPE_COMPACT=0, E_PPE_CUT_PLAN=0).  Appends the "kernel med" lines to OUTDIR/summary.txt.
set -o pipefail
O=gpurun_out/$1; C=$2; shift 2
mkdir -p $O
V=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=(--variant "$1"); shift; done
[ "$1" = "--" ] && shift
timeout -k 10 600 python -u tools/ab_bench.py --config $C "${V[@]}" "$@" > $O/ab_$C.txt 2>&1 && \
grep "kernel med" $O/ab_$C.txt | sed "s/^/$C /" >> $O/summary.txt
