"""bench.py --config D1's batch construction (CPU, oracle): every timed batch is the same fragment slice with a
different source-address top byte, so its datagrams are all new (no batch meets an earlier one's FCBs) and every
batch does the same reassembly work.  Checked with the oracle's sequential Defrag (tests/test_oracle_defrag.py pins
it to dataplane/src/decode/decode-defrag.c)."""
import numpy as np

import bench
import pyoracle
from ppe import synth


def test_d1_batch_variants_are_independent_and_equivalent():
    n = 3000
    a, o, l = synth.make_fragment_stream(int(n / 3.1) + 64, seed=synth.SEED + 7)
    off, lens = o[:n].copy(), l[:n].copy()
    end = int(off[-1]) + int(lens[-1])
    arena = np.zeros(end + 64, np.uint8)
    arena[:end] = a[:end]
    pos, variant = bench.defrag_batch_variants(arena, off, lens, 3)
    v2, v3 = variant(2), variant(3)
    assert np.array_equal(np.nonzero(v2 != arena)[0], np.unique(pos[arena[pos] != 2]))
    assert (v2[pos] == 2).all() and (v3[pos] == 3).all()
    ids = np.arange(n, dtype=np.uint64)

    def fresh(v):
        d = pyoracle.OracleDefrag(fcb_max=1 << 16)
        try:
            return d.batch(v, off, lens, 100, ids=ids), d.stats()
        finally:
            d.close()

    r2, s2 = fresh(v2)
    r3, s3 = fresh(v3)
    assert np.array_equal(r2["status"], r3["status"]) and r2["n_dgram"] == r3["n_dgram"] > 0
    assert np.array_equal(r2["dgram_len"], r3["dgram_len"])
    # the same table fed both batches: the second behaves as if fresh (no DELETED / chained fragments from the first)
    d = pyoracle.OracleDefrag(fcb_max=1 << 16)
    try:
        d.batch(v2, off, lens, 100, ids=ids)
        r = d.batch(v3, off, lens, 101, ids=ids)
        st = d.stats()
    finally:
        d.close()
    assert np.array_equal(r["status"], r3["status"]) and r["n_dgram"] == r3["n_dgram"]
    assert st["new_fcb"] == 2 * s3["new_fcb"] and st["st_fcb_full"] == 0
