"""GPU forms of the flow-hash steering steps (ppe_steer_partition, ppe_gather_rows, ppe_scatter_rows) against the host
stand-ins of tests/test_steer.py, and the whole steered stateful path with G virtual ranks on one GPU (one engine
context and flow table per rank; the all-to-all exchanges done by tensor slicing) against the owners' oracle tables."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import torch  # noqa: E402

from ppe import Engine, synth  # noqa: E402
from ppe.dist import DeviceSteerOps, steer_finish, steer_prepare  # noqa: E402
from test_steer import expected, make_rank_batch, steer_partition_ref  # noqa: E402

DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    e = Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("n", [1, 63, 64, 1000, 100_003])
@pytest.mark.parametrize("world,rank", [(1, 0), (2, 1), (3, 2), (8, 5), (16, 0)])
def test_partition_kernel(eng, n, world, rank):
    rng = np.random.default_rng(n * 31 + world)
    v = (rng.integers(0, 2, n) * 0x20000).astype(np.uint32)
    h = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    ops = DeviceSteerOps(eng)
    perm, counts = ops.partition(torch.from_numpy(v.view(np.int32)).to(DEV), torch.from_numpy(h.view(np.int32)).to(DEV),
                                 world, rank)
    torch.cuda.synchronize()
    want_perm, want_counts = steer_partition_ref(v, h, world, rank)
    assert np.array_equal(counts.cpu().numpy().view(np.uint32), want_counts)
    assert np.array_equal(perm.cpu().numpy().view(np.uint32), want_perm)


@pytest.mark.parametrize("row", [4, 16, 64, 128])
def test_gather_scatter_rows(eng, row):
    rng = np.random.default_rng(row)
    n = 70_001
    src = rng.integers(0, 256, (n, row), dtype=np.uint8)
    perm = rng.permutation(n).astype(np.int32)
    ops = DeviceSteerOps(eng)
    ts, tp = torch.from_numpy(src).to(DEV), torch.from_numpy(perm).to(DEV)
    g = ops.gather(ts, tp)
    s = ops.scatter(g, tp)
    torch.cuda.synchronize()
    assert np.array_equal(g.cpu().numpy(), src[perm])
    assert np.array_equal(s.cpu().numpy(), src)


@pytest.mark.parametrize("world", [2, 4])
def test_steered_flow_virtual_ranks(world):
    """Every rank's batches through the owners' GPU flow tables, with the exchanges done in-process."""
    rules = synth.make_rules(64, seed=5)
    engs = [Engine(0) for _ in range(world)]
    try:
        ops = []
        for e in engs:
            e.commit(rules, default_action=0)
            e.flow_create(2000, 1 << 14)
            ops.append(DeviceSteerOps(e))
        want = expected(world, rules, 3, 5000)
        for b in range(3):
            cfg = engs[0].cfg(0, 1, 5000 + b)
            prep = []
            for r in range(world):
                pk = make_rank_batch(r, b, rules)
                prep.append(steer_prepare(ops[r], torch.from_numpy(pk["hdr"]).to(DEV),
                                          torch.from_numpy(pk["len"].view(np.int32)).to(DEV), cfg, world, r))
            counts = [p[1].cpu().numpy().astype(np.int64) for p in prep]
            off = [np.concatenate([[0], np.cumsum(c)]) for c in counts]
            res = []
            for own in range(world):  # owner `own` receives source 0's segment first, then source 1's, ...
                hdr = torch.cat([prep[s][2][off[s][own]:off[s][own + 1]] for s in range(world)])
                lens = torch.cat([prep[s][3][off[s][own]:off[s][own + 1]] for s in range(world)])
                res.append(ops[own].classify_flow(hdr, lens, cfg))
            for s in range(world):
                back = torch.cat([res[own][sum(int(counts[x][own]) for x in range(s)):
                                           sum(int(counts[x][own]) for x in range(s + 1))] for own in range(world)])
                out = steer_finish(ops[s], back, prep[s][0])
                torch.cuda.synchronize()
                got = np.stack([out["verdict"].cpu().numpy().view(np.uint32).astype(np.int64),
                                out["flow_hash"].cpu().numpy().view(np.uint32).astype(np.int64),
                                out["acl_hit"].cpu().numpy().astype(np.int64)], 1)
                assert np.array_equal(got, want[s][b]), (b, s)
    finally:
        for e in engs:
            e.close()
