#!/usr/bin/env python3
"""In-process A/B timing of kernel variants (different library builds and/or tunings) on the same resident data,
interleaved over rounds so device clock and thermal drift hit every variant alike (cdna_hip_programming.md §5.4
rule 24).  Prints median / min kernel time and step time per variant.

  python tools/ab_bench.py --config C1 --variant base=packet-process-engine_amd/libppe_hip.so \
      --variant b512=packet-process-engine_amd/libppe_hip.so:block=512
"""
import argparse
import os
import ctypes as C
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "packet-process-engine_amd"), str(ROOT / "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ppe import Engine, abi, synth  # noqa: E402

NOW = 1_700_000_000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C1")
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--stride", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--nbufs", type=int, default=4)
    ap.add_argument("--binth", type=int, default=0)
    ap.add_argument("--variant", action="append", required=True, help="name=libpath[:key=val,...]")
    ap.add_argument("--check", action="store_true", help="compare every variant's outputs with the first")
    ap.add_argument("--reuse", action="store_true",
                    help="diagnostic: keep --nbufs buffers and reuse them within a launch (an on-die packet stream)")
    args = ap.parse_args()
    # every batch of one launch distinct: a launch's batch groups run concurrently (a repeated buffer would be
    # re-read from the Infinity Cache)
    ap_reuse = args.reuse
    if not ap_reuse:
        args.nbufs = max(args.nbufs, args.steps)
    if args.binth:
        import os
        os.environ["PPE_BINTH"] = str(args.binth)

    c = synth.CONFIGS[args.config]
    n = args.n or c["n"]
    rules = synth.make_rules(c["rules"])
    dev = torch.device("cuda:0")
    bufs = []
    gen = [synth.make_packets(n, rules, seed=synth.SEED + 1 + 7919 * g, kind=c["kind"], stride=args.stride)
           for g in range(2)]
    for b in range(args.nbufs):  # 2 generated batches; every buffer its own device allocation
        pk = gen[b % 2]
        hdr = torch.from_numpy(pk["hdr"]).to(dev)
        lens = torch.from_numpy(pk["len"].view(np.int32)).to(dev)
        outs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(5)] + \
               [torch.empty((n + 63) // 64, dtype=torch.int32, device=dev)]
        bufs.append((hdr, lens, outs))
    libs = {}
    variants = []
    for spec in args.variant:
        name, rest = spec.split("=", 1)
        path, _, kv = rest.partition(":")
        path = str(Path(path).resolve())
        if path not in libs:
            libs[path] = abi.load_variant(path)
        kvs = dict(x.split("=") for x in kv.split(",")) if kv else {}
        # E_NAME=value: environment variable NAME set while this variant runs (knobs the engine reads per launch)
        venv = {k[2:]: kvs.pop(k) for k in list(kvs) if k.startswith("E_")}
        import os
        if "pipemode" in kvs:  # ppe_classify_batches stream arrangement (PPE_PIPE_MODE, read at context creation)
            os.environ["PPE_PIPE_MODE"] = kvs.pop("pipemode")
        if "bpl" in kvs:  # ppe_classify_batches: batches per launch (PPE_BATCHES_PER_LAUNCH)
            os.environ["PPE_BATCHES_PER_LAUNCH"] = kvs.pop("bpl")
        os.environ["PPE_GROUPS"] = kvs.pop("groups", "8")  # batch groups of waves (read at context creation)
        os.environ.update(venv)
        eng = Engine(0, lib=libs[path])
        # outs=sep (default): separate FW / DROP lists + tile counts; outs=part: one partition list, no tile counts;
        # outs=part8: the compact partition list (1 B per packet, the bench's layout; ABI version >= 4)
        mode = kvs.pop("outs", "sep")
        # streams=N: consecutive launches round-robin over N streams (batch pipelining: a launch's ramp-up overlaps
        # the previous one's tail); each stream needs its own output buffers, so --nbufs must be a multiple of N
        nstr = int(kvs.pop("streams", "1"))
        # api=batches: the step loop is one ppe_classify_batches call (the engine's own two-stream pipeline)
        api = kvs.pop("api", "classify")
        # jump=N: classifier built with exactly N jump bits (0 = single tree); default: the builder's choice
        import os
        os.environ.pop("PPE_JUMP_BITS", None)
        if "jump" in kvs:
            os.environ["PPE_JUMP_BITS"] = kvs.pop("jump")
        eng.commit(rules, default_action=1)
        os.environ.pop("PPE_JUMP_BITS", None)
        if kvs:
            eng.tuning(**{k: int(v) for k, v in kvs.items()})
        calls = []
        for hdr, lens, outs in bufs:
            bb = abi.Batch(hdr.data_ptr(), lens.data_ptr(), None, n, args.stride)
            ptrs = [o.data_ptr() for o in outs]
            if mode == "part":
                ptrs[4], ptrs[5] = ptrs[3], None
            if mode == "part8":
                rr = abi.Result(ptrs[0], ptrs[1], ptrs[2], None, None, None, None, ptrs[3])
            else:
                rr = abi.Result(*ptrs, None)
            calls.append((bb, rr))
        strs = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(nstr - 1)]
        variants.append(dict(name=name, eng=eng, calls=calls, kern=[], step=[], streams=strs, api=api, env=venv))
        for k in venv:
            os.environ.pop(k, None)
    cfg = Engine.cfg(now_seconds=NOW)
    stream = torch.cuda.current_stream(dev)
    sp = C.c_void_p(stream.cuda_stream)

    def run(v, steps, timed):
        saved = {k: os.environ.get(k) for k in v["env"]}
        os.environ.update(v["env"])
        try:
            run_(v, steps, timed)
        finally:
            for k, x in saved.items():
                if x is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = x

    def run_(v, steps, timed):
        fn, ctx = v["eng"].lib.ppe_classify, v["eng"].ctx
        if timed:  # kernel durations (dispatch timestamps), one stream
            v["eng"].timing(True)
            v["eng"].timing_read(reset=True)
            torch.cuda.synchronize()
            for i in range(steps):
                bb, rr = v["calls"][i % len(v["calls"])]
                assert fn(ctx, C.byref(bb), C.byref(rr), C.byref(cfg), sp) == 0
            kms, nl = v["eng"].timing_read(reset=True)
            v["eng"].timing(False)
            v["kern"].append(kms / nl * 1e3)
        # step time: back-to-back launches without per-launch events, round-robin over the variant's streams
        strs = v["streams"]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(stream)
        for st in strs[1:]:
            st.wait_event(e0)
        if v["api"].startswith("batches"):
            ch = int(v["api"][7:] or steps)  # api=batchesK: K batches per ppe_classify_batches call
            for j in range(0, steps, ch):
                m = min(ch, steps - j)
                ins = (abi.Batch * m)(*(v["calls"][i % len(v["calls"])][0] for i in range(j, j + m)))
                outs = (abi.Result * m)(*(v["calls"][i % len(v["calls"])][1] for i in range(j, j + m)))
                assert v["eng"].lib.ppe_classify_batches(ctx, ins, outs, m, C.byref(cfg), sp) == 0
        else:
            for i in range(steps):
                bb, rr = v["calls"][i % len(v["calls"])]
                st = strs[i % len(strs)]
                assert fn(ctx, C.byref(bb), C.byref(rr), C.byref(cfg), C.c_void_p(st.cuda_stream)) == 0
        for st in strs[1:]:
            ev = torch.cuda.Event()
            ev.record(st)
            stream.wait_event(ev)
        e1.record(stream)
        torch.cuda.synchronize()
        if timed:
            v["step"].append(e0.elapsed_time(e1) / steps * 1e3)

    ref = None
    for v in variants:
        run(v, 3, False)
        if args.check:
            got = [o.cpu().numpy().copy() for o in bufs[0][2]]
            if ref is None:
                ref = got
            else:
                same = all(np.array_equal(a, b) for a, b in zip(ref[:3], got[:3]))
                print(f"{v['name']}: outputs {'identical' if same else 'DIFFER'} to {variants[0]['name']}")
    for r in range(args.rounds):
        order = variants[r % len(variants):] + variants[:r % len(variants)]
        for v in order:
            run(v, args.steps, True)
    res = {}
    for v in variants:
        k, s = v["kern"], v["step"]
        res[v["name"]] = {"kern_med_us": round(statistics.median(k), 3), "kern_min_us": round(min(k), 3),
                          "step_med_us": round(statistics.median(s), 3), "mpps_med": round(n / statistics.median(s), 1),
                          "tuning": v["eng"].tuning(), "launch": v["eng"].launch_info()}
        print(f"{v['name']:>12s}: kernel med {res[v['name']]['kern_med_us']:8.3f} us  min {min(k):8.3f}  "
              f"step med {statistics.median(s):8.3f} us  ({n / statistics.median(s):9.1f} Mpps)  "
              f"{res[v['name']]['launch']}")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
