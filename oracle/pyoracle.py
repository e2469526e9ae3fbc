"""TEST INFRASTRUCTURE ONLY: ctypes binding of the CPU oracle (oracle/liboracle.so) and of the reference's own
flow hash (oracle/_ref/libref_tluhash.so, built from /root/reference when present).  Used by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker — never by the product path."""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
LIB = ORACLE_DIR / "liboracle.so"
REF_LIB = ORACLE_DIR / "_ref" / "libref_tluhash.so"


class OCfg(C.Structure):
    _fields_ = [("unsupport_proto_action", C.c_uint32), ("syn_check", C.c_uint32), ("now_seconds", C.c_uint64)]


class OResult(C.Structure):
    _fields_ = [("status", C.c_uint32), ("action", C.c_uint32), ("flags", C.c_uint32), ("flow_hash", C.c_uint32),
                ("acl_hit", C.c_int32), ("sip", C.c_uint32), ("dip", C.c_uint32), ("sport", C.c_uint32),
                ("dport", C.c_uint32), ("proto", C.c_uint32), ("paylen", C.c_uint32), ("counters", C.c_uint32),
                ("reach", C.c_uint32), ("tcp_ws", C.c_uint32), ("mset", C.c_uint32), ("l3off", C.c_uint32),
                ("l4off", C.c_uint32), ("payoff", C.c_uint32), ("frag_id", C.c_uint32), ("frag_off", C.c_uint32),
                ("frag_len", C.c_uint32), ("opt_past", C.c_uint32)]


# OResult.mset: the mbuf fields the reference's decoders wrote (oracle/ppe_oracle.h ORACLE_M_*)
M_ETH, M_VLAN, M_L3, M_IP, M_FRAG, M_L4H, M_L4, M_WS, M_FLOW = (1 << i for i in range(9))


_lib = None


def load():
    global _lib
    if _lib is None:
        if not LIB.exists():
            raise OSError(f"{LIB} missing: run `make -C oracle`")
        lib = C.CDLL(str(LIB))
        vp, u32, u64 = C.c_void_p, C.c_uint32, C.c_uint64
        lib.oracle_set_rules.argtypes = [vp, vp, u32, u32]
        lib.oracle_set_image.argtypes = [vp, u32]
        lib.oracle_tluhash.argtypes = [u32, u32]
        lib.oracle_tluhash.restype = u32
        lib.oracle_flow_hashfn.argtypes = [u32, u32, u32, u32, u32]
        lib.oracle_flow_hashfn.restype = u32
        lib.oracle_classify.argtypes = [vp, u32, u32, u64, C.POINTER(OCfg), C.POINTER(OResult)]
        lib.oracle_classify_batch.argtypes = [vp, u32, vp, vp, u32, C.POINTER(OCfg), C.c_int, C.c_int, vp, vp, vp,
                                              vp, vp, vp]
        lib.oracle_classify_batch.restype = C.c_int
        lib.oracle_set_pin_cpus.argtypes = [C.POINTER(C.c_int), C.c_int]
        lib.oracle_set_pin_cpus.restype = C.c_int
        lib.oracle_acl_linear.argtypes = [u32, u32, u32, u32, u32, vp, vp, u64, C.POINTER(u32)]
        lib.oracle_acl_linear.restype = C.c_int32
        lib.oracle_acl_tree.argtypes = [u32, u32, u32, u32, u32, vp, vp, u64, C.POINTER(u32)]
        lib.oracle_acl_tree.restype = C.c_int32
        for fn in ("oracle_acl_blocks", "oracle_acl_cut"):
            getattr(lib, fn).argtypes = [u32, u32, u32, u32, u32, vp, vp, u64, C.POINTER(u32)]
            getattr(lib, fn).restype = C.c_int32
        lib.oracle_flow_create.argtypes = [u32]
        lib.oracle_flow_create.restype = vp
        lib.oracle_flow_destroy.argtypes = [vp]
        lib.oracle_flow_classify_batch.argtypes = [vp, vp, u32, vp, vp, u32, C.POINTER(OCfg), C.c_int, vp, vp, vp,
                                                   vp, vp]
        lib.oracle_flow_classify_batch.restype = C.c_int
        lib.oracle_flow_age.argtypes = [vp, u64, u64]
        lib.oracle_flow_age.restype = u64
        lib.oracle_flow_dump.argtypes = [vp, vp, u32]
        lib.oracle_flow_dump.restype = u32
        lib.oracle_flow_stats.argtypes = [vp, C.POINTER(u64), C.POINTER(u64), C.POINTER(u64)]
        lib.oracle_defrag_create.argtypes = [u32, u32, u32, u32]
        lib.oracle_defrag_create.restype = vp
        lib.oracle_defrag_destroy.argtypes = [vp]
        lib.oracle_defrag_batch.argtypes = [vp, vp, vp, vp, vp, u32, u64, vp, vp, vp, vp, vp]
        lib.oracle_defrag_batch.restype = u32
        lib.oracle_defrag_age.argtypes = [vp, u64, u64, vp, u32, C.POINTER(u32)]
        lib.oracle_defrag_age.restype = u32
        lib.oracle_defrag_stats.argtypes = [vp, vp]
        _lib = lib
    return _lib


class Oracle:
    """Holds references to the rule arrays the C oracle points at."""

    def __init__(self, rules=None, used=None, default_action=1, image=None):
        self.lib = load()
        self.set_rules(rules, used, default_action)
        self.image = None
        if image is not None:
            self.set_image(image)

    def set_rules(self, rules, used=None, default_action=1):
        from ppe.abi import RULE_DTYPE
        self.rules = np.ascontiguousarray(rules if rules is not None else np.zeros(0, RULE_DTYPE), RULE_DTYPE)
        self.used = None if used is None else np.ascontiguousarray(used, np.uint8)
        self.lib.oracle_set_rules(self.rules.ctypes.data if len(self.rules) else None,
                                  self.used.ctypes.data if self.used is not None else None, len(self.rules),
                                  int(default_action))

    def set_image(self, image):
        self.image = np.ascontiguousarray(image, np.uint32)
        self.lib.oracle_set_image(self.image.ctypes.data, len(self.image))

    @staticmethod
    def cfg(unsupport_proto_action=0, syn_check=1, now_seconds=0):
        return OCfg(unsupport_proto_action, syn_check, now_seconds)

    def classify_one(self, pkt: bytes, length=None, ts=0, cfg=None) -> dict:
        buf = np.frombuffer(bytes(pkt), np.uint8).copy() if len(pkt) else np.zeros(1, np.uint8)
        r = OResult()
        self.lib.oracle_classify(buf.ctypes.data, len(pkt), len(pkt) if length is None else int(length), int(ts),
                                 C.byref(cfg or self.cfg()), C.byref(r))
        return {k: getattr(r, k) for k, _ in OResult._fields_}

    def pin(self, cpus):
        """Pin classify_batch's shard threads, thread t on cpus[t % len(cpus)] (empty: unpinned)."""
        arr = (C.c_int * max(len(cpus), 1))(*cpus)
        if self.lib.oracle_set_pin_cpus(arr, len(cpus)) != 0:
            raise ValueError("bad cpu list")

    def classify_batch(self, hdr, lens, ts=None, cfg=None, nthreads=1, use_tree=False):
        hdr = np.ascontiguousarray(hdr, np.uint8)
        lens = np.ascontiguousarray(lens, np.uint32)
        n, stride = hdr.shape
        out = dict(verdict=np.zeros(n, np.uint32), flow_hash=np.zeros(n, np.uint32),
                   acl_hit=np.zeros(n, np.int32), tuple=np.zeros((n, 4), np.uint32), reach=np.zeros(n, np.uint32),
                   counters=np.zeros(32, np.uint64))
        if ts is not None:
            ts = np.ascontiguousarray(ts, np.uint64)
        if use_tree and self.image is None:
            raise ValueError("use_tree needs set_image()")
        self.lib.oracle_classify_batch(hdr.ctypes.data, stride, lens.ctypes.data,
                                       ts.ctypes.data if ts is not None else None, n, C.byref(cfg or self.cfg()),
                                       int(nthreads), int(use_tree), out["verdict"].ctypes.data,
                                       out["flow_hash"].ctypes.data, out["acl_hit"].ctypes.data,
                                       out["tuple"].ctypes.data, out["reach"].ctypes.data,
                                       out["counters"].ctypes.data)
        return out




class OracleFlow:
    """One core's flow table (dataplane/src/flow/flow.c) driven by the oracle's FlowHandlePacket, batch by batch in
    packet order; `oracle` supplies the rule set (and image for use_tree)."""

    def __init__(self, oracle: Oracle, capacity=100000):
        self.o = oracle
        self.lib = oracle.lib
        self.h = self.lib.oracle_flow_create(int(capacity))
        if not self.h:
            raise MemoryError("oracle_flow_create")

    def close(self):
        if self.h:
            self.lib.oracle_flow_destroy(self.h)
            self.h = None

    __del__ = close

    def classify_batch(self, hdr, lens, ts=None, cfg=None, use_tree=False):
        hdr = np.ascontiguousarray(hdr, np.uint8)
        lens = np.ascontiguousarray(lens, np.uint32)
        n, stride = hdr.shape
        out = dict(verdict=np.zeros(n, np.uint32), flow_hash=np.zeros(n, np.uint32), acl_hit=np.zeros(n, np.int32),
                   tuple=np.zeros((n, 4), np.uint32), counters=np.zeros(32, np.uint64))
        if ts is not None:
            ts = np.ascontiguousarray(ts, np.uint64)
        self.lib.oracle_flow_classify_batch(self.h, hdr.ctypes.data, stride, lens.ctypes.data,
                                            ts.ctypes.data if ts is not None else None, n,
                                            C.byref(cfg or self.o.cfg()), int(use_tree),
                                            out["verdict"].ctypes.data, out["flow_hash"].ctypes.data,
                                            out["acl_hit"].ctypes.data, out["tuple"].ctypes.data,
                                            out["counters"].ctypes.data)
        return out

    def age(self, now, timeout=20):
        return int(self.lib.oracle_flow_age(self.h, int(now), int(timeout)))

    def dump(self) -> np.ndarray:
        from ppe.abi import FLOW_ENTRY_DTYPE
        n = self.lib.oracle_flow_dump(self.h, None, 0)
        out = np.zeros(n, FLOW_ENTRY_DTYPE)
        self.lib.oracle_flow_dump(self.h, out.ctypes.data if n else None, n)
        return out

    def stats(self) -> dict:
        a, b, c = C.c_uint64(), C.c_uint64(), C.c_uint64()
        self.lib.oracle_flow_stats(self.h, C.byref(a), C.byref(b), C.byref(c))
        return dict(live=a.value, new_flow=b.value, del_flow=c.value)


DF_STATS = ["running", "new_fcb", "del_fcb", "st_cached", "st_reasm", "st_setup_err", "st_fcb_full", "st_hw2sw_err",
            "st_deleted", "st_cache_full", "st_defrag_err", "st_not_frag", "teardrop", "timeout_drop", "datagrams"]


class OracleDefrag:
    """One core's IPv4 reassembly (dataplane/src/decode/decode-defrag.c) restated sequentially in C."""

    def __init__(self, fcb_max=0, cache_max=0, frag_buf=0, reasm_buf=0):
        self.lib = load()
        self.h = self.lib.oracle_defrag_create(fcb_max, cache_max, frag_buf, reasm_buf)
        if not self.h:
            raise MemoryError("oracle_defrag_create")
        self.cache_max = cache_max or 8
        self.reasm_buf = reasm_buf or 8168
        self.fcb_max = fcb_max or 1024

    def close(self):
        if self.h:
            self.lib.oracle_defrag_destroy(self.h)
            self.h = None

    __del__ = close

    def batch(self, pkt, off, lens, now, ids=None, full=True):
        pkt = np.ascontiguousarray(pkt, np.uint8)
        off = np.ascontiguousarray(off, np.uint64)
        lens = np.ascontiguousarray(lens, np.uint32)
        n = len(lens)
        out = dict(status=np.zeros(n, np.uint32), dgram_of=np.zeros(n, np.uint32), dgram_len=np.zeros(n, np.uint32),
                   dgram_frags=np.zeros((n, self.cache_max), np.uint64))
        if full:
            out["dgram_pkt"] = np.zeros((n, self.reasm_buf), np.uint8)
        if ids is not None:
            ids = np.ascontiguousarray(ids, np.uint64)
        nd = self.lib.oracle_defrag_batch(self.h, pkt.ctypes.data, off.ctypes.data, lens.ctypes.data,
                                          ids.ctypes.data if ids is not None else None, n, int(now),
                                          out["status"].ctypes.data, out["dgram_of"].ctypes.data,
                                          out["dgram_pkt"].ctypes.data if full else None, out["dgram_len"].ctypes.data,
                                          out["dgram_frags"].ctypes.data)
        out["n_dgram"] = int(nd)
        return out

    def age(self, now, timeout=20):
        cap = self.fcb_max * self.cache_max
        ids = np.zeros(cap, np.uint64)
        nf = C.c_uint32(0)
        nd = self.lib.oracle_defrag_age(self.h, int(now), int(timeout), ids.ctypes.data, cap, C.byref(nf))
        return ids[:min(nd, cap)], nf.value

    def stats(self) -> dict:
        v = np.zeros(len(DF_STATS), np.uint64)
        self.lib.oracle_defrag_stats(self.h, v.ctypes.data)
        return {k: int(x) for k, x in zip(DF_STATS, v)}


def ref_hash_lib():
    """The reference's own flow_hashfn (tluhash.h compiled unmodified), or None when not built here."""
    if not REF_LIB.exists():
        return None
    lib = C.CDLL(str(REF_LIB))
    lib.ref_flow_hashfn.argtypes = [C.c_uint8, C.c_uint32, C.c_uint32, C.c_uint16, C.c_uint16]
    lib.ref_flow_hashfn.restype = C.c_uint32
    lib.ref_TluHash.argtypes = [C.c_uint32, C.c_uint32]
    lib.ref_TluHash.restype = C.c_uint32
    lib.ref_flow_hashfn_batch.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
    return lib
