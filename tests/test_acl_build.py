"""The host classifier compiler (product code, runs without a GPU): walking its image must give exactly the
linear first-match result for every packet, across rule-set shapes."""
import numpy as np
import pytest

import pyoracle
from ppe import abi, synth
from ppe.abi import RULE_DTYPE

NOW = 1_700_000_000


def compare(rules, used, pk, default_action=1, binth=0, cfg=None):
    img, st = abi.build_image(rules, used, default_action, binth)
    o = pyoracle.Oracle(rules, used, default_action=default_action, image=img)
    cfg = cfg or o.cfg(0, 1, NOW)
    lin = o.classify_batch(pk["hdr"], pk["len"], ts=pk.get("ts"), cfg=cfg, nthreads=4)
    tree = o.classify_batch(pk["hdr"], pk["len"], ts=pk.get("ts"), cfg=cfg, nthreads=4, use_tree=True)
    # the image's 2-level block section (what the multi-tile kernel walks) must give the same answers, and so must its
    # cut lists (image v8: what the cut-list kernel reads) when it has them
    blocks = o.classify_batch(pk["hdr"], pk["len"], ts=pk.get("ts"), cfg=cfg, nthreads=4, use_tree=2)
    cut = o.classify_batch(pk["hdr"], pk["len"], ts=pk.get("ts"), cfg=cfg, nthreads=4, use_tree=3) if img[22] else lin
    for k in ("verdict", "acl_hit", "flow_hash", "counters"):
        assert np.array_equal(lin[k], tree[k]), k
        assert np.array_equal(lin[k], blocks[k]), k
        assert np.array_equal(lin[k], cut[k]), k
    return img, st, lin


@pytest.mark.parametrize("binth", [1, 2, 4, 16])
@pytest.mark.parametrize("nrules,resid", [(16, 0.0), (256, 0.0), (300, 0.3), (1024, 0.1)])
def test_tree_equals_linear(nrules, resid, binth):
    rules = synth.make_rules(nrules, seed=nrules + binth, resid_frac=resid, any_ip_frac=0.1)
    pk = synth.make_packets(6000, rules, seed=5, kind="imix", stride=128, malformed_frac=0.05, with_ts=True)
    img, st, lin = compare(rules, None, pk, binth=binth)
    assert st["n_rules"] == nrules
    assert st["max_depth"] < 60
    assert (lin["acl_hit"] >= 0).sum() > 500


def test_golden_rules_tree(golden):
    pk = {"hdr": golden["hdr"], "len": golden["len"], "ts": golden["ts"]}
    for binth in (1, 4):
        _, _, lin = compare(golden["rules"], golden["used"], pk, binth=binth)
        assert np.array_equal(lin["verdict"], golden["a_verdict"])


def test_heavily_overlapping_wildcards():
    rng = np.random.default_rng(3)
    n = 400
    r = np.zeros(n, RULE_DTYPE)
    r["sip_mask"] = rng.choice([0, 8, 16], n)
    r["sip"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32) & 0xFFFF0000
    r["dip_mask"] = rng.choice([0, 4], n)
    r["dip"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    lo = rng.integers(0, 60000, n)
    r["dport_start"], r["dport_end"] = lo, lo + rng.integers(0, 5000, n)
    r["sport_end"] = 65535
    r["protocol_start"], r["protocol_end"] = 0, 255
    r["action"] = rng.integers(0, 2, n)
    pk = synth.make_packets(8000, r, seed=9, stride=128, hit_frac=0.9)
    compare(r, None, pk, default_action=0)


def test_default_action_and_empty_set():
    pk = synth.make_packets(2000, np.zeros(0, RULE_DTYPE), seed=2, stride=128)
    for da in (0, 1):
        img, st, lin = compare(np.zeros(0, RULE_DTYPE), None, pk, default_action=da)
        assert st["n_nodes"] == 1 and (lin["acl_hit"] == -1).all()


def test_used_mask_and_empty_ranges():
    rules = synth.make_rules(200, seed=4)
    rules["sport_start"][::7] = 60000
    rules["sport_end"][::7] = 10  # empty: never matches
    used = (np.arange(200) % 5 != 0).astype(np.uint8)
    pk = synth.make_packets(5000, rules, seed=8, stride=128)
    _, st, _ = compare(rules, used, pk)
    assert st["n_rules"] == int(((np.arange(200) % 5 != 0) & (np.arange(200) % 7 != 0)).sum())


def test_bad_mask_rejected():
    rules = synth.make_rules(4)
    rules["sip_mask"][2] = 33
    with pytest.raises(ValueError):
        abi.build_image(rules)


def test_large_ruleset_builds_bounded():
    rules = synth.make_rules(65536)
    img, st = abi.build_image(rules, default_action=1, binth=1)
    assert st["n_rules"] == 65536 and st["max_depth"] < 60
    assert len(img) * 4 == st["blob_bytes"] < 64 << 20
    pk = synth.make_packets(3000, rules, seed=1, stride=128)
    o = pyoracle.Oracle(rules, default_action=1, image=img)
    lin = o.classify_batch(pk["hdr"], pk["len"], cfg=o.cfg(0, 1, NOW), nthreads=8)
    tree = o.classify_batch(pk["hdr"], pk["len"], cfg=o.cfg(0, 1, NOW), nthreads=8, use_tree=True)
    assert np.array_equal(lin["acl_hit"], tree["acl_hit"])


def test_image_layout():
    """Image format v8 (csrc/ppe_image.h): optional jump table after the 32-word header, 16-B nodes {threshold, left,
    right, child key slots}, leaves as walk fixed points, the always-matching sentinel rule at slot n_rules, the
    2-level block section, the compact records after it (one candidate per leaf, no residual rules), then the cut
    lists (32-B aligned header, groups, entries)."""
    for nrules in (64, 256):
        rules = synth.make_rules(nrules)
        img, st = abi.build_image(rules)
        assert img[0] == 0x41455050 and img[1] == 8
        assert img[2] == st["n_nodes"] and img[4] == nrules and img[11] == len(img)
        assert img[7] % 8 == 0  # rules 32-B aligned
        off = int(img[5])
        jw = int(img[14])
        nroots = 1
        if jw:  # jump root: 2^bits bucket entries -> subtree roots (the first nodes), with their key slots
            dim, shift, bits = jw & 0xFF, (jw >> 8) & 0xFF, (jw >> 16) & 0xFF
            assert dim <= 4 and 1 <= bits <= 16 and off == 32 + (1 << bits)
            width = 32 if dim <= 1 else (16 if dim <= 3 else 8)
            assert shift == width - bits
            jt = img[32:off]
            roots = (jt & 0xFFFFFF).astype(np.int64)
            assert (np.diff(roots) >= 0).all() and roots[0] == 4 * off  # runs of buckets, in order
            nroots = len(np.unique(roots))
            assert roots[-1] == 4 * off + 16 * (nroots - 1)
        nodes = img[off:off + 4 * img[2]].reshape(-1, 4)
        own = 4 * off + 16 * np.arange(len(nodes))
        is_leaf = nodes[:, 0] == 0xFFFFFFFF
        leaves, inner = nodes[is_leaf], nodes[~is_leaf]
        if jw:
            assert ((jt >> 24) == np.where(is_leaf[(roots - 4 * off) // 16], 5, (jt >> 24))).all()
        assert img[12] == 1  # binth 1: one candidate per leaf
        assert (leaves[:, 1] == own[is_leaf]).all()  # a leaf's left child is itself (walk fixed point)
        assert (leaves[:, 3] == (5 << 8 | 5 << 24)).all()  # ... and its key slot is the zero key
        assert (leaves[:, 2] <= nrules).all()  # payload: a rule slot or the sentinel (n_rules)
        # internal: children are the two consecutive nodes after it (BFS), after every root
        li = (inner[:, 1] - 4 * off) // 16
        assert ((inner[:, 2] - 4 * off) // 16 == li + 1).all() and (li > np.nonzero(~is_leaf)[0]).all()
        assert (li >= nroots).all()
        # a child's key slot (carried by its parent) is 5 exactly for leaves
        ks_l, ks_r = (inner[:, 3] >> 8) & 0xFF, (inner[:, 3] >> 24) & 0xFF
        assert ((ks_l == 5) == is_leaf[li]).all() and ((ks_r == 5) == is_leaf[li + 1]).all()
        assert (ks_l <= 5).all() and (ks_r <= 5).all() and (img[13] >> 8) <= 5
        sent = img[img[7] + 8 * nrules: img[7] + 8 * (nrules + 1)]
        assert sent[1] == sent[3] == sent[5] == 0xFFFFFFFF and sent[7] == 0x1FFFFFFF
        # block section: after the residual records, its jump table (root block = root node index), 32-B blocks;
        # every non-leaf exit names a later block, every block but the roots is named exactly once
        ob, nb, oblk = int(img[15]), int(img[16]), int(img[17])
        oc, oi = int(img[19]), int(img[20])
        oct_ = int(img[22])
        assert oc == oblk + 8 * nb and oi == 0 and oct_ == (oc + 4 * (nrules + 1) + 7) // 8 * 8  # compact, no holes
        h = cut_header(img)
        assert h["slc"] == oct_ + 16 and h["gbase"] == h["slc"] + 4 * h["groups"] and h["fp"] == h["gbase"] + h["groups"]
        assert h["ent"] % 32 == 0 and h["fp"] + (h["entries"] + 7) // 8 + 2 <= h["ent"] < h["fp"] + (h["entries"] + 7) // 8 + 34
        # (a cut that fits LDS: dense lines of 8 entries, the 16-bit ids after them)
        assert h["ids16"] and not h["lines_ids"] and h["epl"] == 8 and h["div"] == 1 << 29
        assert h["off_id"] == h["ent"] + 32 * h["lines"] and h["off_id"] + (h["entries"] + 1) // 2 == len(img)
        assert ob >= int(img[8]) and ob % 8 == 0 and oblk % 8 == 0
        if jw:
            assert np.array_equal(img[ob:ob + (1 << bits)].astype(np.int64), (roots - 4 * off) // 16)
        blk = img[oblk:oc].reshape(nb, 8)
        ex = blk[:, 4:].astype(np.int64)
        inner_ex = ex[(ex & 0x80000000) == 0]
        assert np.array_equal(np.sort(inner_ex), np.arange(nroots, nb))
        leaf_ex = ex[(ex & 0x80000000) != 0]
        slot = leaf_ex & 0xFFFFFF
        assert (slot <= nrules).all()
        assert (((leaf_ex >> 29) & 1) == (slot == nrules)).all()  # NOHIT exactly on the sentinel
        crec = img[oc:oc + 4 * (nrules + 1)].reshape(nrules + 1, 4)
        assert np.array_equal(crec[nrules], [0x80000000, 0x80000000, 0, 0xFFFFFFFF])


def test_long_leaf_list_escape():
    """More than 254 candidates in one leaf (rules the 5-tuple cannot separate: same box, different MACs) use the
    escaped count word; the walk must still find the lowest matching index."""
    n = 600
    rules = np.zeros(n, RULE_DTYPE)
    rules["sip"] = 0x0A000000
    rules["sip_mask"] = 8
    rules["sport_end"] = rules["dport_end"] = 0xFFFF
    rules["protocol_end"] = 0xFF
    rules["action"] = np.arange(n) & 1
    macs = np.arange(1, n + 1, dtype=np.uint64)
    for b in range(6):
        rules["dmac"][:, b] = (macs >> np.uint64(8 * b)) & np.uint64(0xFF)
    img, st = abi.build_image(rules, default_action=1)
    nodes = img[img[5]:img[5] + 4 * img[2]].reshape(-1, 4)
    leaves = nodes[nodes[:, 0] == 0xFFFFFFFF]
    assert ((leaves[:, 2] >> 24) == 255).any() and img[12] >= n
    pk = synth.make_packets(4000, rules, seed=5, kind="udp64", stride=64)
    # point some packets' dmac at late rules
    idx = np.arange(0, 4000, 7)
    want = (idx * 13) % n
    for b in range(6):
        pk["hdr"][idx, b] = ((want + 1) >> (8 * b)) & 0xFF
    o = pyoracle.Oracle(rules, default_action=1, image=img)
    tree = o.classify_batch(pk["hdr"], pk["len"], nthreads=8, use_tree=True)
    lin = o.classify_batch(pk["hdr"], pk["len"], nthreads=8)
    assert np.array_equal(tree["acl_hit"], lin["acl_hit"])
    assert (lin["acl_hit"] >= 300).any()


@pytest.mark.parametrize("jump", ["0", "4", "8", "12"])
@pytest.mark.parametrize("nrules,resid,any_ip", [(256, 0.0, 0.0), (300, 0.3, 0.2), (2048, 0.05, 0.1)])
def test_jump_root_equals_linear(monkeypatch, jump, nrules, resid, any_ip):
    """Image v4 jump root (a cut of the top bits of one dimension, one subtree per run of buckets): forced to each
    width, the walk still gives exactly the linear first match — wildcard rules replicated into every bucket,
    residual MAC / time rules, prefixes shorter than the cut."""
    monkeypatch.setenv("PPE_JUMP_BITS", jump)
    rules = synth.make_rules(nrules, seed=nrules + int(jump), resid_frac=resid, any_ip_frac=any_ip)
    pk = synth.make_packets(6000, rules, seed=11, kind="imix", stride=128, malformed_frac=0.02, with_ts=True)
    img, st, lin = compare(rules, None, pk)
    jw = int(img[14])
    assert (jw >> 16) & 0xFF == int(jump) and (jump == "0") == (jw == 0)
    assert (lin["acl_hit"] >= 0).sum() > 500


@pytest.mark.parametrize("compact", ["1", "0"])
def test_compact_leaves_edge_cases(monkeypatch, compact):
    """Compact leaf exits and 16-B records (image v6) against the linear definition: prefix lengths 0, 1, 31 and 32
    (the /32 flag), protocol ranges containing 6 and / or 17 or neither (only TCP / UDP reach the ACL), actions other
    than 0 / 1 (only DROP drops), unused entries (the slot → index table), default FW and DROP; and the same rules
    built without compact leaves (PPE_COMPACT=0, the v5 leaf path)."""
    monkeypatch.setenv("PPE_COMPACT", compact)
    rng = np.random.default_rng(77)
    n = 1500
    r = synth.make_rules(n, seed=78)
    r["sip_mask"] = rng.choice([0, 1, 2, 8, 24, 30, 31, 32], n)
    r["dip_mask"] = rng.choice([0, 1, 16, 31, 32], n)
    pr = rng.integers(0, 6, n)
    r["protocol_start"] = np.choose(pr, [6, 17, 0, 5, 7, 18])
    r["protocol_end"] = np.choose(pr, [6, 17, 255, 7, 16, 255])
    r["action"] = rng.choice([0, 1, 2, 0xFFFF], n)
    used = (rng.random(n) < 0.8).astype(np.uint8)
    for da in (0, 1):
        pk = synth.make_packets(8000, r, seed=79 + da, kind="imix", stride=128, malformed_frac=0.02, hit_frac=0.9)
        img, st, lin = compare(r, used, pk, default_action=da)
        assert (int(img[19]) != 0) == (compact == "1") and (int(img[20]) != 0) == (compact == "1")
        assert (lin["acl_hit"] >= 0).sum() > 2000
        # every protocol kind and prefix kind is hit
        hit = lin["acl_hit"][lin["acl_hit"] >= 0]
        assert len(np.unique(pr[hit])) >= 4 and (r["sip_mask"][hit] == 32).any() and (r["sip_mask"][hit] == 0).any()


@pytest.mark.parametrize("nrules,resid,binth", [(256, 0.0, 1), (2048, 0.0, 1), (300, 0.3, 1), (1024, 0.0, 4)])
def test_blocks_equal_linear(nrules, resid, binth):
    """The 2-level blocks (image word 21) walk to the same leaves as the node tree: compact leaves, leaf lists
    (binth 4) and residual rules, jump root on."""
    rules = synth.make_rules(nrules, seed=nrules + 7, resid_frac=resid, any_ip_frac=0.1)
    pk = synth.make_packets(6000, rules, seed=12, kind="imix", stride=128, malformed_frac=0.02, with_ts=True)
    img, st, lin = compare(rules, None, pk, binth=binth)
    assert int(img[21]) == 2
    assert int(img[17]) % 8 == 0 and (lin["acl_hit"] >= 0).sum() > 500


def test_default_block_levels_and_lds_fit():
    """2-level blocks by default (3-level ones measured slower on C3); C4's block section with its compact
    records (4,096 rules) fits a 1024-thread workgroup's LDS whole."""
    img2, _ = abi.build_image(synth.make_rules(4096))
    assert int(img2[21]) == 2
    assert (int(img2[22]) - int(img2[15])) * 4 <= 158 * 1024  # the block section and records end where the cut starts


def cut_header(img):
    h = int(img[22])
    return dict(b0=int(img[h]) & 0xFF, b1=(int(img[h]) >> 8) & 0xFF, ids16=bool(int(img[h]) & 0x10000),
                lines_ids=bool(int(img[h]) & 0x20000), off_id=int(img[h + 12]),
                buckets=int(img[h + 1]), entries=int(img[h + 2]), max_len=int(img[h + 3]), slc=int(img[h + 4]),
                ent=int(img[h + 5]), groups=int(img[h + 6]), epl=int(img[h + 7]), gbase=int(img[h + 8]),
                fp=int(img[h + 9]), div=int(img[h + 10]), lines=int(img[h + 11]))


def cut_entries(img, h):
    """The entries (n x 4 words) and rule ids of the image's 128-B entry lines (ids in-line, or the id array)."""
    lines = np.asarray(img[h["ent"]:h["ent"] + 32 * h["lines"]], np.uint32).reshape(-1, 32)
    epl = h["epl"]
    ent = lines[:, : 4 * epl].reshape(-1, 4)[: h["entries"]]
    if h["lines_ids"]:
        tail = lines[:, 4 * epl:]
        ids = (tail.view(np.uint16)[:, :epl] if h["ids16"] else tail[:, :epl]).reshape(-1)
    else:
        arr = np.asarray(img[h["off_id"]:], np.uint32)
        ids = arr.view(np.uint16) if h["ids16"] else arr
    return ent, ids[: h["entries"]].astype(np.int64)


def cut_lengths(img, h):
    """Each bucket's list length from the bit-sliced groups."""
    sl = np.asarray(img[h["slc"]:h["slc"] + 4 * h["groups"]], np.uint32).reshape(-1, 4)
    b = np.arange(h["buckets"])
    return sum(((sl[b >> 5, i] >> (b & 31)) & 1).astype(np.int64) << i for i in range(4))


@pytest.mark.parametrize("lines", ["0", "1"])
@pytest.mark.parametrize("bits", ["5", "6", "8", "11", "16"])
def test_cut_lists_equal_linear(monkeypatch, bits, lines):
    """The cut lists (image v8) at every width, forced by PPE_CUT_BITS, against the linear definition: prefix lengths
    0 / 1 / 7 / 8 / 31 / 32 (rules replicated into the buckets they meet, lists closed after a rule that covers the
    whole bucket), any-port rules, protocol ranges with and without 6 / 17, actions other than 0 / 1, unused
    entries, default FW and DROP, with the ids in the entry lines and in their own array (PPE_CUT_LINES).  The image's
    group table encodes each bucket's list exactly."""
    monkeypatch.setenv("PPE_CUT_BITS", bits)
    monkeypatch.setenv("PPE_CUT_LINES", lines)
    rng = np.random.default_rng(1234 + int(bits))
    n = {5: 80, 6: 120}.get(int(bits), 700)  # (every list within 15 entries)
    r = synth.make_rules(n, seed=90 + int(bits))
    r["sip_mask"] = rng.choice([0, 1, 7, 8, 16, 31, 32], n, p=[0.02, 0.03, 0.1, 0.25, 0.3, 0.15, 0.15])
    r["dip_mask"] = rng.choice([0, 1, 8, 24, 32], n, p=[0.02, 0.03, 0.35, 0.3, 0.3])
    anyport = rng.random(n) < 0.3
    for f in ("sport", "dport"):
        r[f + "_start"][anyport] = 0
        r[f + "_end"][anyport] = 65535
    pr = rng.integers(0, 4, n)
    r["protocol_start"] = np.choose(pr, [6, 17, 0, 7])
    r["protocol_end"] = np.choose(pr, [6, 17, 255, 16])
    r["action"] = rng.choice([0, 1, 2], n)
    used = (rng.random(n) < 0.9).astype(np.uint8)
    for da in (0, 1):
        pk = synth.make_packets(6000, r, seed=91 + da, kind="imix", stride=128, malformed_frac=0.02, hit_frac=0.9)
        img, st, lin = compare(r, used, pk, default_action=da)
        assert int(img[22]) != 0, "cut lists expected"
        h = cut_header(img)
        assert h["b0"] + h["b1"] == int(bits) and h["b0"] >= 3 and h["b1"] >= 2
        assert st["cut_bits"] == h["b0"] | h["b1"] << 8
        assert h["buckets"] == 1 << int(bits) and h["groups"] == max(1, h["buckets"] // 32)
        # the groups' lengths add up to the entries, each at most 15, and the group bases are their prefix sums
        lens = cut_lengths(img, h)
        assert lens.sum() == h["entries"] == st["cut_entries"] and lens.max() == h["max_len"] <= 15
        gb = np.asarray(img[h["gbase"]:h["gbase"] + h["groups"]], np.int64)
        assert np.array_equal(gb, np.concatenate([[0], np.cumsum(lens)])[: h["groups"] * 32 : 32])
        assert (lin["acl_hit"] >= 0).sum() > 1000
        # each entry's DROP flag (sip word bit 1) is its rule's action; 16-bit ids (every index < 2^16)
        ent, ids = cut_entries(img, h)
        assert h["lines_ids"] == (lines == "1")
        epl = 7 if h["lines_ids"] else 8
        assert h["ids16"] and h["epl"] == epl and h["lines"] == -(-h["entries"] // epl) and h["ent"] % 32 == 0
        assert np.array_equal((ent[:, 0] >> 1) & 1, (np.asarray(r["action"])[ids] == 1).astype(np.uint32))


def test_cut_lists_rule_indices_above_32767():
    """40,000 rules, half of them unused: 20,000 in the image but indices up to 39,999, which the 16-bit id words
    hold whole (the DROP flag lives in the entry); the cut walk equals the linear definition."""
    n = 40_000
    rng = np.random.default_rng(77)
    r = synth.make_rules(n, seed=78)
    r["action"] = rng.choice([0, 1, 2], n)
    used = (rng.random(n) < 0.5).astype(np.uint8)
    pk = synth.make_packets(20000, r, seed=79, stride=64, hit_frac=0.8)
    img, st, lin = compare(r, used, pk, default_action=1)
    h = cut_header(img)
    assert h["ids16"] and h["entries"] > 0
    _, ids = cut_entries(img, h)
    assert ids.max() >= 32768 and used[ids].all()
    assert (lin["acl_hit"] >= 32768).sum() > 1000


def test_cut_lists_rejected_or_absent(monkeypatch):
    """No cut lists for rule sets with MAC / time fields (the classify kernel's cut check has none), none when
    every width leaves a bucket with more than 15 candidates (then the kernel walks the tree), and none below 5 bits
    (b0 >= 3 and b1 >= 2 keep the flag bits free below the relative prefixes)."""
    img, st = abi.build_image(synth.make_rules(300, seed=3, resid_frac=0.3))
    assert int(img[22]) == 0 and st["cut_entries"] == 0
    monkeypatch.setenv("PPE_CUT_BITS", "4")
    img, st = abi.build_image(synth.make_rules(8, seed=3))
    assert int(img[22]) == 0
    monkeypatch.delenv("PPE_CUT_BITS")
    r = synth.make_rules(40, seed=5)
    r["sip_mask"] = 0
    r["dip_mask"] = 0  # 40 overlapping wildcard-address rules: every bucket holds all 40
    r["sport_start"] = np.arange(40) * 100
    r["sport_end"] = np.arange(40) * 100 + 50
    img, st = abi.build_image(r)
    assert int(img[22]) == 0
    pk = synth.make_packets(3000, r, seed=6, stride=128, hit_frac=0.9)
    compare(r, None, pk)


def test_cut_lists_of_the_bench_rule_sets():
    """C3's 65,536 rules (every prefix /8 or longer): a 16-bit cut of 8 sip and 8 dip bits, no replication, at most
    15 entries per bucket, 16-bit ids; C4's 4,096 rules: a 12-bit cut, whose groups, 16-B entries and 16-bit ids fit
    half a CU's LDS.  Both walks equal the linear definition."""
    for nrules, seed, bits in ((65536, 0x5EED, 16), (4096, 0x5EED, 12)):
        rules = synth.make_rules(nrules)
        img, st = abi.build_image(rules)
        h = cut_header(img)
        assert h["b0"] + h["b1"] == bits and h["entries"] <= nrules and h["max_len"] <= 15, h
        assert nrules == 4096 or (h["b0"], h["b1"]) == (8, 8)
        assert h["ids16"]
        # C3 reads its entries from L2: ids in the lines; C4's cut fits LDS: dense entries and the id array
        assert h["lines_ids"] == (nrules == 65536)
        if nrules == 4096:
            assert (len(img) - h["slc"]) * 4 + 3 * 1024 <= 80 * 1024  # groups .. ids in half the LDS
        pk = synth.make_packets(20000, rules, seed=seed + 1, stride=64)
        o = pyoracle.Oracle(rules, None, default_action=1, image=img)
        lin = o.classify_batch(pk["hdr"], pk["len"], cfg=o.cfg(0, 1, NOW), nthreads=8)
        cut = o.classify_batch(pk["hdr"], pk["len"], cfg=o.cfg(0, 1, NOW), nthreads=8, use_tree=3)
        for k in ("verdict", "acl_hit", "counters"):
            assert np.array_equal(lin[k], cut[k]), k


@pytest.mark.parametrize("lines", ["0", "1"])
def test_cut_lists_32bit_rule_ids(monkeypatch, lines):
    """used rule indices past 65,535 (a sparse `used` array over 400,000 slots, the extended API's range)
    switch the cut lists to 32-bit ids (6 entries per line with the ids in the lines, or the 32-bit id array); the
    cut walk over that layout equals the linear definition, with the ids in the lines and in their own array."""
    monkeypatch.setenv("PPE_CUT_LINES", lines)
    base = synth.make_rules(4096, seed=73)
    slots = 400_000
    rules = np.zeros(slots, RULE_DTYPE)
    used = np.zeros(slots, np.uint8)
    pos = np.unique(np.concatenate([np.sort(np.random.default_rng(74).choice(np.arange(1, slots), 4093,
                                                                               replace=False)),
                                    [65_536, 131_071, slots - 1]]))
    rules[pos] = base[:len(pos)]
    used[pos] = 1
    pk = synth.make_packets(20000, base[:len(pos)], seed=75, stride=64, hit_frac=0.9)
    img, st, lin = compare(rules, used, pk, default_action=1)
    assert int(img[22]) != 0, "cut lists expected"
    h = cut_header(img)
    assert not h["ids16"] and h["lines_ids"] == (lines == "1")
    if h["lines_ids"]:
        assert h["epl"] == 6
    _, ids = cut_entries(img, h)
    assert ids.max() > 65_535 and used[ids].all()
    assert (lin["acl_hit"] > 65_535).sum() > 1000
