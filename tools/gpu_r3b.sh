# round 3: GPU suite, smoke, default bench line, then the same stateless configs with compact leaves off (A/B)
set -o pipefail
O=gpurun_out/${1:-r3b}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err && \
PPE_COMPACT=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive --stateful "" > $O/bench_nocompact.json 2> $O/bench_nocompact.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive --stateful "" > $O/bench2.json 2> $O/bench2.err &&
# the select-form tuple zeroing (round-2 dport-0 miscompile) rebuilt as a variant: the PART-variant test against it
PPE_LIB=packet-process-engine_amd/libppe_hip_sel.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "partition_layout or exact_workload" > $O/pytest_sel.txt 2>&1
