#!/usr/bin/env python3
"""Profiling driver (diagnostics): `--calls` ppe_defrag calls over distinct D1 fragment batches (bench.py's D1
workload: every batch with fresh datagrams), nothing else on the GPU, so rocprofv3 --pmc passes see exactly those
calls' kernels (tools/collect_traffic.py --kernel ppe_defrag --calls K sums them per call).

  python tools/defrag_run.py --calls 8
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "packet-process-engine_amd"), str(ROOT / "oracle"), str(ROOT)]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ppe import Defrag, Engine, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=8)
    a = ap.parse_args()
    import bench
    cfgd = synth.CONFIGS["D1"]
    n = cfgd["n"]
    a_full, o_full, l_full = synth.make_fragment_stream(int(n / 3.1) + 64, seed=synth.SEED + 7)
    off, lens = o_full[:n].copy(), l_full[:n].copy()
    end = int(off[-1]) + int(lens[-1])
    arena = np.zeros(end + 64, np.uint8)
    arena[:end] = a_full[:end]
    pos, _ = bench.defrag_batch_variants(arena, off, lens, a.calls)
    dev = torch.device("cuda:0")
    eng = Engine(0)
    d = Defrag(eng, fcb_max=cfgd["fcb_max"])
    t_off = torch.from_numpy(off.view(np.int64)).to(dev)
    t_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    t_ids = torch.arange(n, dtype=torch.int64, device=dev)
    base = torch.from_numpy(arena).to(dev)
    t_pos = torch.from_numpy(pos).to(dev)
    out = d.alloc_out(n, 128)
    pkts = []
    for v in range(a.calls):
        t = base.clone()
        t[t_pos] = v + 2
        pkts.append(t)
    torch.cuda.synchronize()
    for v in range(a.calls):
        d.run_torch(pkts[v], t_off, t_len, out, bench.NOW, ids=t_ids)
    torch.cuda.synchronize()
    # algorithmic bytes of one call, as bench.py run_defrag counts them
    n_dgram = int(out["n_dgram"].item())
    dlen = int(out["dgram_len"][:n_dgram].to(torch.int64).sum().item())
    st = out["status"].cpu().numpy().view(np.uint32) & 0xff
    fr_ids = out["dgram_frags"][:n_dgram].cpu().numpy().view(np.uint64).ravel()
    stored = np.isin(st, (0, 1, 2))
    stored[fr_ids[fr_ids < n].astype(np.int64)] = False
    cm = d.info_["cache_max"]
    alg = (float(lens.astype(np.int64).sum()) + float(lens[stored].astype(np.int64).sum()) + 2.0 * dlen +
           n_dgram * (128 + 4 + 8 * cm) + n * 28.0)
    print(f"defrag calls {a.calls} fragments per call {n} alg_bytes_per_call {alg:.0f}")
    d.close()
    eng.close()


if __name__ == "__main__":
    main()
