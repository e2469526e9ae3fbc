#!/usr/bin/env python3
"""Regenerate ref_rule_v1.npz (run in the build container: needs oracle/_ref/libref_rule.so, which oracle/Makefile
builds from the reference's own rule/rule.c + ipc/msgque.c, unmodified, when /root/reference is present).

The fuzzed corpus of tests/rule_corpus.py ('@' rule files with edge values of every scanf conversion, Rule_add /
Rule_del_by_id / Rule_duplicate_check / Rule_del_all sequences, FULL at 10,000) is run through the REFERENCE's rule
store and parser; the return codes and every resulting rule_list_t image are frozen, so tests/test_rules.py checks the
product's csrc/rule_store.c against the reference's behaviour byte for byte without the reference tree (GPU box).

Fixture arrays: corpus (JSON: cases + reference results), hdr (56-B list header per case), idx / ent / off (every
entry with a nonzero byte: index, its 61 bytes, per-case offsets)."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path[:0] = [str(HERE.parent)]

import rule_corpus as rc  # noqa: E402

SEED = 20261018


def main():
    so = ROOT / "oracle" / "_ref" / "libref_rule.so"
    if not so.exists():
        sys.exit(f"{so} missing: run `make -C oracle ref` with /root/reference present")
    ref = C.CDLL(str(so))
    assert ref.ref_rule_list_size() == rc.LIST_BYTES
    cases = rc.make_corpus(SEED)
    out = rc.Runner(ref, "ref").run(cases)
    results = [r for r, _ in out]
    hdr, idx, ent, off = rc.pack_images([im for _, im in out])
    corpus = np.frombuffer(rc.dumps(cases, results).encode(), np.uint8)
    np.savez_compressed(HERE / "ref_rule_v1.npz", corpus=corpus, hdr=hdr, idx=idx, ent=ent, off=off)
    n_ok = sum(1 for ops, r in zip(cases, results) for o, x in zip(ops, r) if o[0] == "file" and x and x[-1] == 0)
    print(f"ref_rule_v1.npz: {len(cases)} cases, {sum(len(c) for c in cases)} ops, {n_ok} files loaded to the end, "
          f"{len(idx)} stored entries")


if __name__ == "__main__":
    main()
