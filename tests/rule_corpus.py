"""Rule-store / '@' rule-file corpus shared by tests/golden/gen_rule_golden.py (which runs it through the reference's
own rule/rule.c + ipc/msgque.c, compiled unmodified into oracle/_ref/libref_rule.so) and tests/test_rules.py (which
runs it through the product's csrc/rule_store.c and compares).

A case is a list of operations on one fresh rule list (Rule_list_init's state, srv_rule.c:82-86):
  ("file", text)     the reference caller's loop, srv_rule.c:783-794: while (!feof(fp)) { ret = Rule_Load_Line(fp,
                     line); if (ret) break; line++; } -> the list of return codes
  ("add", tuple)     Rule_add(tuple, &id) -> (rc, id)            (60-B RCP_BLOCK_ACL_RULE_TUPLE, hex)
  ("del", id)        Rule_del_by_id(id) -> rc                    (id < RULE_ENTRY_MAX: the reference does not check)
  ("dup", tuple)     Rule_duplicate_check(tuple) -> rc
  ("delall",)        Rule_del_all() -> rc
After the case, the whole rule_list_t (610,056 B on x86-64) is compared byte for byte."""
from __future__ import annotations

import ctypes as C
import json
import os
import tempfile

import numpy as np

RULE_ENTRY_MAX = 10000
LIST_BYTES = 56 + 61 * RULE_ENTRY_MAX
TUPLE_BYTES = 60


# ---- '@' line fuzz: each field mostly valid, sometimes an edge of the reference's scanf conversions ----

def _pick(rng, good, edge, p_edge):
    return str(edge[rng.integers(len(edge))]) if rng.random() < p_edge else good()


def _mac(rng, p):
    good = lambda: ":".join(f"{int(x):02x}" for x in (rng.integers(0, 256, 6) if rng.random() < 0.4 else [0] * 6))  # noqa: E731
    edge = ["0:1:2:3:4:5", "AB:cd:EF:01:23:45", "abc:0:0:0:0:0", "0x:1:2:3:4:5", "-1:0:0:0:0:0", "+f:0:0:0:0:0",
            "00:00:00:00:00", "00-00-00-00-00-00", "ff:ff:ff:ff:ff:fff", "g0:00:00:00:00:00", "7:7:7:7:7:7"]
    return _pick(rng, good, edge, p)


_BIG = ["4294967295", "4294967296", "4294967297", "2147483647", "2147483648", "-1", "-2147483648", "-2147483649",
        "9223372036854775807", "9223372036854775808", "18446744073709551615", "18446744073709551616",
        "-9223372036854775809", "99999999999999999999999"]


def _ip(rng, p):
    def good():
        if rng.random() < 0.2:
            return "0.0.0.0/0"
        o = rng.integers(0, 256, 4)
        return f"{o[0]}.{o[1]}.{o[2]}.{o[3]}/{int(rng.integers(0, 33))}"
    edge = ["0.0.0.0/8", "1.0.0.0/33", "1.0.0.0/32", "0.0.0.0/-1", "256.0.0.1/8", "1.2.3.300/24", "-1.0.0.0/8",
            "4294967296.0.0.1/8", "1.2.3/8", "1.2.3.4 /8", "1.2.3.4/ 8", "1.2.3.4-8", "1.2.3.4//8", "10.0.0.1/"]
    edge += [f"10.0.0.1/{b}" for b in _BIG] + [f"{b}.0.0.0/8" for b in _BIG[:8]]
    return _pick(rng, good, edge, p)


def _range(rng, p, hi):
    def good():
        a = int(rng.integers(0, hi + 1))
        b = int(rng.integers(a, hi + 1))
        return f"{a} : {b}"
    edge = ["9 : 1", "0:65535", "5 :5", "5: 5", "-1 : 5", "0 : -1", "70000 : 1", "65616 : 65616", "5 - 6", "5 ; 6",
            "256 : 255", "0 : 256", "273 : 273", "1 :", ": 1"] + [f"0 : {b}" for b in _BIG] + [f"{b} : {b}" for b in _BIG]
    return _pick(rng, good, edge, p)


def _time(rng, p):
    good = lambda: "0 0" if rng.random() < 0.6 else f"{int(rng.integers(0, 2**31))} {int(rng.integers(0, 2**31))}"  # noqa: E731
    edge = ["-1 5", "0x10 0", "1700000000 1700000100", "5 4", "18446744073709551615 0", "9223372036854775808 1",
            "-9223372036854775809 0", "1.5 2", "0"]
    return _pick(rng, good, edge, p)


def _int01(rng, p):
    good = lambda: str(int(rng.integers(0, 2)))  # noqa: E731
    edge = ["2", "-1", "65536", "65537", "-65535", "-65536", "131073", "1.5", "x", "01", "+1", "- 1"] + _BIG
    return _pick(rng, good, edge, p)


def rule_line(rng, p=0.08):
    f = [_mac(rng, p), _mac(rng, p), _ip(rng, p), _ip(rng, p), _range(rng, p, 65535), _range(rng, p, 65535),
         _range(rng, p, 255), _time(rng, p), _int01(rng, p), _int01(rng, p)]
    sep = " " if rng.random() < 0.9 else ("\t", "  ", "\n")[int(rng.integers(3))]
    return "@" + (" " if rng.random() < 0.9 else "") + sep.join(f)


def rule_file(rng):
    lines = []
    for _ in range(int(rng.integers(1, 7))):
        r = rng.random()
        if r < 0.1:
            lines.append("# a comment line with no at-sign")
        elif r < 0.15:
            lines.append("junk before the rule " + rule_line(rng))
        elif r < 0.2 and lines:
            lines.append(lines[-1])      # a duplicate line: Rule_add's EXIST, ignored by Rule_Load_Line
        else:
            lines.append(rule_line(rng))
        if rng.random() < 0.1:
            lines[-1] += " " + rule_line(rng)   # two rules on one line
    text = "\n".join(lines)
    r = rng.random()
    if r < 0.1:
        text = text[: int(rng.integers(1, len(text) + 1))]   # EOF inside a rule
    elif r < 0.55:
        text += "\n"
    return text if text.strip("\n") else "#\n"    # (never empty: the reference reads an uninitialised char then)


def rand_tuple(rng, base=None):
    t = bytearray(rng.integers(0, 256, TUPLE_BYTES, dtype=np.uint8).tobytes()) if base is None else bytearray(base)
    if base is not None:
        t[int(rng.integers(TUPLE_BYTES))] ^= 1 << int(rng.integers(8))
    return bytes(t)


def make_corpus(seed: int, n_files: int = 300, n_api: int = 24, full: bool = True) -> list:
    rng = np.random.default_rng(seed)
    cases = []
    for _ in range(n_files):
        ops = [("file", rule_file(rng))]
        if rng.random() < 0.3:
            ops.append(("file", rule_file(rng)))    # a second file on top (its rules add to the list)
        cases.append(ops)
    # the reference caller's full reload: delete all, then the file
    for _ in range(8):
        cases.append([("file", rule_file(rng)), ("delall",), ("file", rule_file(rng))])
    for _ in range(n_api):
        ops, pool = [], []
        for _ in range(int(rng.integers(10, 80))):
            r = rng.random()
            if r < 0.45 or not pool:
                t = rand_tuple(rng, pool[int(rng.integers(len(pool)))] if pool and rng.random() < 0.3 else None)
                if pool and rng.random() < 0.15:
                    t = pool[int(rng.integers(len(pool)))]          # exact duplicate: EXIST
                pool.append(t)
                ops.append(("add", t.hex()))
            elif r < 0.7:
                ops.append(("del", int(rng.integers(0, min(RULE_ENTRY_MAX, len(pool) + 3)))))
            elif r < 0.9:
                ops.append(("dup", pool[int(rng.integers(len(pool)))].hex() if rng.random() < 0.7
                             else rand_tuple(rng).hex()))
            elif r < 0.95:
                ops.append(("delall",))
            else:
                ops.append(("file", rule_file(rng)))
        cases.append(ops)
    if full:
        # FULL at 10,000 (the count check comes before the duplicate check, rule/rule.c:356-368), then frees and
        # first-free reuse, and a file loaded into a full list (Rule_add's FULL is ignored by Rule_Load_Line)
        ops = [("add", (i.to_bytes(4, "little") * 15).hex()) for i in range(RULE_ENTRY_MAX)]
        ops += [("add", (5).to_bytes(4, "little").hex() * 15), ("add", rand_tuple(rng).hex()),
                ("dup", (5).to_bytes(4, "little").hex() * 15), ("file", rule_file(rng))]
        ops += [("del", i) for i in (9999, 0, 5000, 5000)]
        ops += [("add", rand_tuple(rng).hex()) for _ in range(4)]
        ops += [("file", "@ 00:00:00:00:00:00 00:00:00:00:00:00 1.0.0.0/8 0.0.0.0/0 0 : 1 0 : 1 0 : 1 0 0 1 0\n")]
        cases.append(ops)
    return cases


# ---- running a corpus through one library (the reference's or the product's) ----

class Runner:
    """Drives one library's rule store: `lib` exports Rule_* and either ref_rule_list_init/… (the reference
    harness) or ppe_rule_list_init/… (the product); FILE* handles come from libc, which both libraries use."""

    def __init__(self, lib, prefix: str):
        self.lib = lib
        self.init = getattr(lib, prefix + "_rule_list_init")
        self.free = getattr(lib, prefix + "_rule_list_free")
        vp = C.c_void_p
        lib.Rule_Load_Line.argtypes = [vp, C.c_int]
        lib.Rule_Load_Line.restype = C.c_int
        lib.Rule_add.argtypes = [vp, C.POINTER(C.c_uint32)]
        lib.Rule_del_by_id.argtypes = [C.c_uint32]
        lib.Rule_duplicate_check.argtypes = [vp]
        self.libc = C.CDLL(None)
        self.libc.fopen.restype = vp
        self.libc.fopen.argtypes = [C.c_char_p, C.c_char_p]
        self.libc.feof.argtypes = [vp]
        self.libc.fclose.argtypes = [vp]

    def image(self) -> bytes:
        p = C.c_void_p.in_dll(self.lib, "rule_list").value
        return C.string_at(p, LIST_BYTES)

    def run_case(self, ops, tmpdir) -> tuple[list, bytes]:
        self.free()
        assert self.init() == 0
        res = []
        for op in ops:
            kind = op[0]
            if kind == "file":
                path = os.path.join(tmpdir, "rule_config")
                with open(path, "wb") as f:
                    f.write(op[1].encode("latin-1"))
                fp = self.libc.fopen(path.encode(), b"r")
                assert fp
                rcs, line = [], 0
                while not self.libc.feof(fp):
                    rc = self.lib.Rule_Load_Line(fp, line)
                    rcs.append(rc)
                    if rc != 0:
                        break
                    line += 1
                self.libc.fclose(fp)
                res.append(rcs)
            elif kind == "add":
                t = C.create_string_buffer(bytes.fromhex(op[1]), TUPLE_BYTES)
                rid = C.c_uint32(0xFFFFFFFF)
                rc = self.lib.Rule_add(t, C.byref(rid))
                res.append([rc, rid.value])
            elif kind == "del":
                res.append(self.lib.Rule_del_by_id(op[1]))
            elif kind == "dup":
                res.append(self.lib.Rule_duplicate_check(C.create_string_buffer(bytes.fromhex(op[1]), TUPLE_BYTES)))
            elif kind == "delall":
                res.append(self.lib.Rule_del_all())
            else:
                raise ValueError(kind)
        img = self.image()
        self.free()
        return res, img

    def run(self, cases):
        with tempfile.TemporaryDirectory() as d:
            return [self.run_case(ops, d) for ops in cases]


# ---- compact fixture form: the 56-B header plus every entry with a nonzero byte ----

def pack_images(images):
    hdr = np.stack([np.frombuffer(im[:56], np.uint8) for im in images])
    idx, ent, off = [], [], [0]
    for im in images:
        e = np.frombuffer(im[56:], np.uint8).reshape(RULE_ENTRY_MAX, 61)
        nz = np.nonzero(e.any(axis=1))[0]
        idx.append(nz.astype(np.uint16))
        ent.append(e[nz])
        off.append(off[-1] + len(nz))
    return hdr, np.concatenate(idx), np.concatenate(ent), np.array(off, np.int64)


def unpack_image(hdr, idx, ent, off, k) -> bytes:
    e = np.zeros((RULE_ENTRY_MAX, 61), np.uint8)
    e[idx[off[k]:off[k + 1]]] = ent[off[k]:off[k + 1]]
    return hdr[k].tobytes() + e.tobytes()


def dumps(cases, results) -> str:
    return json.dumps({"cases": cases, "results": results})
