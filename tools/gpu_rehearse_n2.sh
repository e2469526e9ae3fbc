# N > 1 rehearsal on a one-GPU box: bench.py --gpus 2 spawns 2 ranks (torch.distributed.run), both on cuda:0, gloo for
# the barriers / MAX reduction; every rank runs its own resident batches, parity samples and roofline launch
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u bench.py --gpus 2 --shared-gpu --steps 16 --warmup 2 --no-cpu-baseline --configs C4 \
  --no-host-inclusive > $O/bench_n2.json 2> $O/bench_n2.err || exit 1
timeout -k 10 400 python -u bench.py --gpus 2 --shared-gpu --scaling strong --steps 8 --warmup 2 --configs "" \
  --no-cpu-baseline --no-host-inclusive > $O/bench_n2_strong.json 2> $O/bench_n2_strong.err
