"""ctypes view of the C ABI in include/ppe_hip.h / ppe_acl.h (test and bench plumbing — the product is the C ABI).

The library is loaded from the package tree (``packet-process-engine_amd/libppe_hip.so``); a missing library raises
immediately: there is no Python or CPU fallback for any classification.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent.parent          # packet-process-engine_amd/
REPO_DIR = PKG_DIR.parent
LIB_PATH = PKG_DIR / "libppe_hip.so"

# ---- constants mirrored from include/ppe_hip.h ----
PPE_OK = 0
ST = dict(ACL_FW=0, ACL_DROP=1, L2_HEADER_ERR=2, L2_UNSUPPORT=3, VLAN_HEADER_ERR=4, VLAN_LAYER_EXCEED=5,
          VLAN_UNSUPPORT=6, IPV4_HEADER_ERR=7, IPV4_VERSION_ERR=8, IPV4_LEN_ERR=9, FRAG_LEN_ERR=10, FRAG=11,
          IPV4_UNSUPPORT=12, UDP_HEADER_ERR=13, UDP_LEN_ERR=14, TCP_HEADER_ERR=15, TCP_LEN_ERR=16,
          FLOW_TCP_NO_SYN_FIRST=17, WINDOW_PUNT=18, FLOW_NOMEM=19)
ST_NAME = {v: k for k, v in ST.items()}
ACT_FW, ACT_DROP, ACT_PUNT = 0, 1, 2
F_VLAN, F_L4, F_TCP, F_SYN, F_ACL, F_FRAG = 0x1, 0x2, 0x4, 0x8, 0x10, 0x20
F_FLOW, F_TOCLIENT, F_NEWFLOW = 0x40, 0x80, 0x100
COUNTERS = ["l2_headerlen_err", "l2_unsupport", "l2_rx_ok",
            "vlan_headerlen_err", "vlan_layer_exceed", "vlan_unsupport", "vlan_rx_ok",
            "ipv4_headerlen_err", "ipv4_version_err", "ipv4_pktlen_err", "ipv4_unsupport", "ipv4_rx_ok",
            "frag_fraglen_err", "frag_punt",
            "udp_headerlen_err", "udp_pktlen_err", "udp_rx_ok",
            "tcp_headerlen_err", "tcp_pktlen_err", "tcp_rx_ok",
            "acl_drop", "acl_fw",
            "flow_proc_ok", "flow_proc_fail", "flow_tcp_no_syn_first",
            "out_fw", "out_drop", "out_punt", "window_punt", "pkts", "flow_node_nomem", "rx_bytes"]
ACL_RULE_ACTION_FW, ACL_RULE_ACTION_DROP = 0, 1
RULE_ENTRY_MAX = 10000

# RCP_BLOCK_ACL_RULE_TUPLE, include/rpc-common.h:97-114 (packed, 60 bytes)
RULE_DTYPE = np.dtype([
    ("time_start", "<u8"), ("time_end", "<u8"), ("smac", "u1", 6), ("dmac", "u1", 6),
    ("sport_start", "<u2"), ("sport_end", "<u2"), ("sip", "<u4"), ("dip", "<u4"),
    ("sip_mask", "<u4"), ("dip_mask", "<u4"), ("dport_start", "<u2"), ("dport_end", "<u2"),
    ("protocol_start", "u1"), ("protocol_end", "u1"), ("action", "<u2"), ("logable", "<u4"),
])
assert RULE_DTYPE.itemsize == 60


class Batch(C.Structure):
    _fields_ = [("hdr", C.c_void_p), ("len", C.c_void_p), ("ts", C.c_void_p), ("n", C.c_uint32),
                ("stride", C.c_uint32)]


class Result(C.Structure):
    _fields_ = [("verdict", C.c_void_p), ("flow_hash", C.c_void_p), ("acl_hit", C.c_void_p),
                ("fw_idx", C.c_void_p), ("drop_idx", C.c_void_p), ("tile_cnt", C.c_void_p), ("tuple", C.c_void_p),
                ("part8", C.c_void_p),  # compact partition list (ABI version 4)
                ("packed", C.c_void_p)]  # 8-B verdict + flow hash + ACL hit (ABI version 8)


PACKED_MAX_RULES = (1 << 19) - 1  # include/ppe_hip.h PPE_PACKED_MAX_RULES


def unpack(packed: np.ndarray) -> dict:
    """The packed result words (ppe_result_t.packed, PPE_PACKED_* in include/ppe_hip.h) as the three SoA outputs:
    verdict (status | action << 8 | flags << 16), flow_hash and acl_hit."""
    x = np.ascontiguousarray(packed).view(np.uint64)
    hi = (x >> np.uint64(32)).astype(np.uint32)
    verdict = (hi & 31) | (((hi >> 5) & 3) << 8) | (((hi >> 7) & 63) << 16)
    return {"verdict": verdict.astype(np.uint32), "flow_hash": (x & np.uint64(0xFFFFFFFF)).astype(np.uint32),
            "acl_hit": ((hi >> 13).astype(np.int64) - 1).astype(np.int32)}


class Cfg(C.Structure):
    _fields_ = [("unsupport_proto_action", C.c_uint32), ("syn_check", C.c_uint32), ("now_seconds", C.c_uint64)]


class AclStats(C.Structure):
    _fields_ = [("n_rules", C.c_uint32), ("n_nodes", C.c_uint32), ("n_leaves", C.c_uint32),
                ("n_leaf_entries", C.c_uint32), ("max_depth", C.c_uint32), ("avg_depth", C.c_double),
                ("blob_bytes", C.c_uint32), ("lds_resident", C.c_uint32), ("build_ms", C.c_double),
                ("cut_bits", C.c_uint32), ("cut_entries", C.c_uint32)]  # ABI version 6

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Counters(C.Structure):
    _fields_ = [("c", C.c_uint64 * 32)]

    def as_dict(self):
        return {name: int(self.c[i]) for i, name in enumerate(COUNTERS)}


class Tuning(C.Structure):
    _fields_ = [("block", C.c_uint32), ("blocks_per_cu", C.c_uint32), ("pipeline", C.c_uint32),
                ("lds_image", C.c_uint32), ("batches_per_launch", C.c_uint32)]

    def __init__(self, block=0, blocks_per_cu=0, pipeline=0, lds_image=1, batches_per_launch=0):
        super().__init__(block, blocks_per_cu, pipeline, lds_image, batches_per_launch)

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class FlowInfo(C.Structure):
    _fields_ = [("live", C.c_uint64), ("new_flow", C.c_uint64), ("del_flow", C.c_uint64), ("capacity", C.c_uint32),
                ("max_batch", C.c_uint32), ("slots", C.c_uint32), ("tombstones", C.c_uint32), ("rehashes", C.c_uint32),
                ("pad", C.c_uint32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "pad"}


# ppe_flow_entry_t (include/ppe_hip.h), 64 bytes
FLOW_ENTRY_DTYPE = np.dtype([("sip", "<u4"), ("dip", "<u4"), ("sport", "<u2"), ("dport", "<u2"), ("protocol", "u1"),
                             ("pad", "u1", 3), ("flowflags", "<u4"), ("slot", "<u4"), ("pktcnts2d", "<u8"),
                             ("pktcntd2s", "<u8"), ("bytecnts2d", "<u8"), ("bytecntd2s", "<u8"),
                             ("last_seen", "<u8")])
assert FLOW_ENTRY_DTYPE.itemsize == 64


class Tuples(C.Structure):
    _fields_ = [("tuple", C.c_void_p), ("macs", C.c_void_p), ("ts", C.c_void_p), ("n", C.c_uint32)]


# ---- IPv4 reassembly (ppe_defrag_*) ----
DF = dict(CACHED=0, REASM=1, SETUP_ERR=2, FCB_FULL=3, HW2SW_ERR=4, DELETED=5, CACHE_FULL=6, DEFRAG_ERR=7, NOT_FRAG=8)
DF_NAME = {v: k for k, v in DF.items()}
DF_TEARDROP = 0x100


class DefragCfg(C.Structure):
    _fields_ = [("fcb_max", C.c_uint32), ("cache_max", C.c_uint32), ("frag_buf_bytes", C.c_uint32),
                ("reasm_buf_bytes", C.c_uint32), ("max_batch", C.c_uint32), ("pad", C.c_uint32)]


class FragBatch(C.Structure):
    _fields_ = [("pkt", C.c_void_p), ("off", C.c_void_p), ("len", C.c_void_p), ("id", C.c_void_p),
                ("n", C.c_uint32), ("pad", C.c_uint32), ("now_seconds", C.c_uint64)]


class DefragOut(C.Structure):
    _fields_ = [("status", C.c_void_p), ("dgram_of", C.c_void_p), ("dgram_hdr", C.c_void_p),
                ("dgram_len", C.c_void_p), ("dgram_pkt", C.c_void_p), ("dgram_frags", C.c_void_p),
                ("n_dgram", C.c_void_p), ("hdr_stride", C.c_uint32), ("pad", C.c_uint32)]


class DefragInfo(C.Structure):
    _fields_ = [("running", C.c_uint64), ("new_fcb", C.c_uint64), ("del_fcb", C.c_uint64),
                ("st", C.c_uint64 * 9), ("teardrop", C.c_uint64), ("timeout_drop", C.c_uint64),
                ("datagrams", C.c_uint64), ("fcb_max", C.c_uint32), ("cache_max", C.c_uint32),
                ("frag_buf_bytes", C.c_uint32), ("reasm_buf_bytes", C.c_uint32), ("max_batch", C.c_uint32),
                ("slots", C.c_uint32)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_ if k != "st"}
        d.update({"st_" + DF_NAME[i].lower(): int(self.st[i]) for i in range(9)})
        return d


class TCPOpt(C.Structure):  # include/ppe_decode.h (decode-tcp.h:24-28)
    _fields_ = [("type", C.c_uint8), ("len", C.c_uint8), ("data", C.c_void_p)]


class TCPVars(C.Structure):  # decode-tcp.h:34-46: one option slot and the window-scale pointer
    _fields_ = [("tcp_opts", TCPOpt * 1), ("ws", C.c_void_p)]


class Mbuf(C.Structure):
    """include/ppe_decode.h mbuf_t: the reference's mbuf_t field order (dataplane/src/include/mbuf.h:23-87) plus the
    engine's appended results."""
    _fields_ = [("magic_flag", C.c_uint32), ("pkt_space", C.c_uint8), ("flow_log", C.c_uint8),
                ("frag_len", C.c_uint16), ("packet_ptr", C.c_uint64), ("next", C.c_void_p), ("pkt_ptr", C.c_void_p),
                ("ethh", C.c_void_p), ("vlanh", C.c_void_p), ("network_header", C.c_void_p),
                ("transport_header", C.c_void_p), ("input_port", C.c_uint32), ("eth_dst", C.c_uint8 * 6),
                ("eth_src", C.c_uint8 * 6), ("sip", C.c_uint32), ("dip", C.c_uint32), ("sport", C.c_uint16),
                ("dport", C.c_uint16), ("proto", C.c_uint8), ("vlan_idx", C.c_uint8), ("payload_len", C.c_uint16),
                ("vlan_id", C.c_uint16), ("defrag_id", C.c_uint16), ("timestamp", C.c_uint64),
                ("payload", C.c_void_p), ("tcpvars", TCPVars), ("frag_offset", C.c_uint16),
                ("tcp_reasm_overlap", C.c_uint16), ("pkt_totallen", C.c_uint32), ("flags", C.c_uint32),
                ("fcb_hash", C.c_uint32), ("fcb", C.c_void_p), ("fragments", C.c_void_p), ("flow", C.c_void_p),
                ("tcp_seg_raw", C.c_void_p), ("tcp_seg_raw_tail", C.c_void_p), ("tcp_seg_reassem", C.c_void_p),
                ("alState", C.c_void_p), ("FreeState", C.c_void_p), ("tag", C.c_uint32),
                ("ppe_verdict", C.c_uint32), ("ppe_flow_hash", C.c_uint32), ("ppe_acl_hit", C.c_int32),
                ("user", C.c_void_p)]


MBUF_MAGIC_NUM = 0xAB00AB00
TUPLE_OPT_PAST = 1 << 15  # include/ppe_hip.h PPE_TUPLE_OPT_PAST (tuple word 3)


# every symbol include/*.h declares (checked by tests/test_abi.py)
EXPORTS = [
    # ppe_hip.h
    "ppe_abi_version", "ppe_ctx_create", "ppe_ctx_destroy", "ppe_ctx_device", "ppe_rules_commit", "ppe_rules_stage", "ppe_rules_publish", "ppe_classify",
    "ppe_classify_batches", "ppe_classify_host", "ppe_acl_lookup", "ppe_acl_lookup_host", "ppe_dev_alloc", "ppe_dev_free",
    "ppe_host_alloc", "ppe_host_free", "ppe_memcpy_h2d", "ppe_memcpy_d2h", "ppe_memset_d", "ppe_sync",
    "ppe_counters_read", "ppe_counters_clear", "ppe_timing_enable", "ppe_timing_read", "ppe_acl_image",
    "ppe_launch_info", "ppe_last_error", "ppe_acl_build_image", "ppe_acl_free_image", "ppe_set_tuning",
    "ppe_get_tuning", "ppe_flow_create", "ppe_flow_destroy", "ppe_classify_flow", "ppe_flow_age", "ppe_flow_info",
    "ppe_flow_clear_stat", "ppe_flow_dump", "ppe_format_pkt_stat", "ppe_format_flow_stat",
    "ppe_format_pkt_stat_ex", "ppe_format_flow_stat_ex",
    "ppe_steer_partition", "ppe_gather_rows", "ppe_scatter_rows",
    "ppe_defrag_create", "ppe_defrag_destroy", "ppe_defrag", "ppe_defrag_age", "ppe_defrag_info",
    "ppe_defrag_last_error",
    # ppe_acl.h
    "ppe_rule_list_init", "ppe_rule_list_free", "Rule_add", "Rule_del_by_id", "Rule_del_all",
    "Rule_duplicate_check", "Rule_Load_Line", "ppe_rule_load_file", "DP_Acl_Rule_Init", "DP_Acl_Load_Rule",
    "DP_Acl_Rule_Clean", "DP_Acl_Rule_Release", "DP_Acl_Rule_Commit",
    # ppe_decode.h
    "ppe_set_output_hooks", "Decode", "Decode_Flush", "Decode_Set_Burst", "DP_Acl_Lookup_Burst", "DP_Acl_Lookup",
    "reg_fw_alert", "DP_Log_Func", "ppe_compat_ctx",
]
EXPORTED_DATA = ["rule_list", "dp_acl_action_default", "gWstDepth", "gAvgDepth", "gChildCount", "gNumTreeNode",
                 "gNumLeafNode", "unsupport_proto_action", "syn_check", "plugin_modules", "g_acltree_1", "g_acltree_2",
                 "g_acltree_running", "acltree_running_rwlock"]

_lib = None


ABI_VERSION = 8  # include/ppe_hip.h PPE_ABI_VERSION


def load(path: str | os.PathLike | None = None) -> C.CDLL:
    """Load libppe_hip.so (raises OSError if it was not built — no fallback)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else Path(os.environ.get("PPE_LIB", LIB_PATH))
    lib = _open(p, C.RTLD_GLOBAL)
    if lib.ppe_abi_version() != ABI_VERSION:  # structs below would not match the library's
        raise OSError(f"{p}: ABI version {lib.ppe_abi_version()}, this binding expects {ABI_VERSION} (rebuild)")
    if path is None:
        _lib = lib
    return lib


def load_variant(path: str | os.PathLike) -> C.CDLL:
    """Load another build of the library side by side (RTLD_LOCAL), for in-process A/B timing."""
    return _open(Path(path), C.RTLD_LOCAL, strict=False)


def _open(p: Path, mode, strict: bool = True) -> C.CDLL:
    if not p.exists():
        raise OSError(f"{p} not found: build it with `make -C packet-process-engine_amd` (no CPU fallback exists)")
    lib = C.CDLL(str(p), mode=mode)
    vp, u32, i32, u64 = C.c_void_p, C.c_uint32, C.c_int32, C.c_uint64
    sig = {
        "ppe_abi_version": ([], C.c_int),
        "ppe_ctx_create": ([C.c_int, C.POINTER(vp)], C.c_int),
        "ppe_ctx_destroy": ([vp], C.c_int),
        "ppe_ctx_device": ([vp], C.c_int),
        "ppe_rules_commit": ([vp, vp, vp, u32, u32, C.POINTER(AclStats)], C.c_int),
        "ppe_rules_stage": ([vp, vp, vp, u32, u32, C.POINTER(AclStats), C.POINTER(C.c_uint64)], C.c_int),
        "ppe_rules_publish": ([vp, C.c_uint64], C.c_int),
        "ppe_classify": ([vp, C.POINTER(Batch), C.POINTER(Result), C.POINTER(Cfg), vp], C.c_int),
        "ppe_classify_host": ([vp, C.POINTER(Batch), C.POINTER(Result), C.POINTER(Cfg), u32], C.c_int),
        "ppe_classify_batches": ([vp, C.POINTER(Batch), C.POINTER(Result), u32, C.POINTER(Cfg), vp], C.c_int),
        "ppe_acl_lookup": ([vp, C.POINTER(Tuples), vp, vp, u64, vp], C.c_int),
        "ppe_acl_lookup_host": ([vp, C.POINTER(Tuples), vp, vp, u64], C.c_int),
        "ppe_dev_alloc": ([vp, C.c_size_t], vp),
        "ppe_dev_free": ([vp, vp], None),
        "ppe_host_alloc": ([vp, C.c_size_t], vp),
        "ppe_host_free": ([vp, vp], None),
        "ppe_memcpy_h2d": ([vp, vp, vp, C.c_size_t], C.c_int),
        "ppe_memcpy_d2h": ([vp, vp, vp, C.c_size_t], C.c_int),
        "ppe_memset_d": ([vp, vp, C.c_int, C.c_size_t], C.c_int),
        "ppe_sync": ([vp], C.c_int),
        "ppe_counters_read": ([vp, C.POINTER(Counters)], C.c_int),
        "ppe_counters_clear": ([vp], C.c_int),
        "ppe_timing_enable": ([vp, C.c_int], C.c_int),
        "ppe_timing_read": ([vp, C.POINTER(C.c_double), C.POINTER(u32), C.c_int], C.c_int),
        "ppe_acl_image": ([vp, vp, C.POINTER(u32)], C.c_int),
        "ppe_launch_info": ([vp, C.POINTER(u32), C.POINTER(u32), C.POINTER(u32), C.POINTER(u32)], C.c_int),
        "ppe_last_error": ([vp], C.c_char_p),
        "ppe_set_tuning": ([vp, C.POINTER(Tuning)], C.c_int),
        "ppe_get_tuning": ([vp, C.POINTER(Tuning)], C.c_int),
        "ppe_acl_build_image": ([vp, vp, u32, u32, u32, C.POINTER(C.POINTER(u32)), C.POINTER(u32),
                                 C.POINTER(AclStats)], C.c_int),
        "ppe_acl_free_image": ([C.POINTER(u32)], None),
        "ppe_flow_create": ([vp, u32, u32], C.c_int),
        "ppe_flow_destroy": ([vp], C.c_int),
        "ppe_classify_flow": ([vp, C.POINTER(Batch), C.POINTER(Result), C.POINTER(Cfg), vp], C.c_int),
        "ppe_flow_age": ([vp, u64, u64, C.POINTER(u64)], C.c_int),
        "ppe_flow_info": ([vp, C.POINTER(FlowInfo)], C.c_int),
        "ppe_flow_clear_stat": ([vp], C.c_int),
        "ppe_flow_dump": ([vp, vp, u32, C.POINTER(u32)], C.c_int),
        "ppe_format_pkt_stat": ([C.POINTER(Counters), C.c_char_p, C.c_size_t], C.c_int),
        "ppe_steer_partition": ([vp, vp, vp, u32, u32, u32, vp, vp, vp], C.c_int),
        "ppe_gather_rows": ([vp, vp, u32, vp, u32, vp, vp], C.c_int),
        "ppe_scatter_rows": ([vp, vp, u32, vp, u32, vp, vp], C.c_int),
        "ppe_format_flow_stat": ([C.POINTER(FlowInfo), C.c_char_p, C.c_size_t], C.c_int),
        "ppe_format_pkt_stat_ex": ([C.POINTER(Counters), C.POINTER(DefragInfo), C.c_int, C.c_char_p, C.c_size_t],
                                   C.c_int),
        "ppe_format_flow_stat_ex": ([C.POINTER(FlowInfo), C.POINTER(DefragInfo), C.c_char_p, C.c_size_t], C.c_int),
        "ppe_defrag_create": ([vp, C.POINTER(DefragCfg), C.POINTER(vp)], C.c_int),
        "ppe_defrag_destroy": ([vp], C.c_int),
        "ppe_defrag": ([vp, C.POINTER(FragBatch), C.POINTER(DefragOut), vp], C.c_int),
        "ppe_defrag_age": ([vp, u64, u64, vp, u32, C.POINTER(u32), C.POINTER(u32)], C.c_int),
        "ppe_defrag_info": ([vp, C.POINTER(DefragInfo)], C.c_int),
        "ppe_defrag_last_error": ([vp], C.c_char_p),
        "ppe_rule_list_init": ([], C.c_int),
        "ppe_rule_list_free": ([], None),
        "Rule_add": ([vp, C.POINTER(u32)], C.c_int),
        "Rule_del_by_id": ([u32], C.c_int),
        "Rule_del_all": ([], C.c_int),
        "Rule_duplicate_check": ([vp], C.c_int),
        "ppe_rule_load_file": ([C.c_char_p], C.c_int),
        "DP_Acl_Rule_Init": ([], C.c_int),
        "DP_Acl_Load_Rule": ([vp, vp, vp], u32),
        "DP_Acl_Rule_Commit": ([], C.c_int),
        "DP_Acl_Rule_Release": ([], None),
        "Decode": ([vp], None),
        "Decode_Flush": ([], C.c_int),
        "Decode_Set_Burst": ([u32], None),
        "DP_Acl_Lookup": ([vp], C.c_int),
        "DP_Acl_Lookup_Burst": ([vp, u32, vp], C.c_int),
    }
    for name, (args, res) in sig.items():
        if not strict and not hasattr(lib, name):  # an older build compared side by side: fewer entry points
            continue
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res
    return lib


def build_image(rules: np.ndarray, used: np.ndarray | None = None, default_action: int = ACL_RULE_ACTION_DROP,
                binth: int = 0):
    """Host-side classifier compiler (no GPU needed): returns (image words as np.uint32, stats dict)."""
    lib = load()
    rules = np.ascontiguousarray(rules, dtype=RULE_DTYPE)
    if used is not None:
        used = np.ascontiguousarray(used, dtype=np.uint8)
    words = C.POINTER(C.c_uint32)()
    nw = C.c_uint32()
    st = AclStats()
    rc = lib.ppe_acl_build_image(rules.ctypes.data if len(rules) else None,
                                 used.ctypes.data if used is not None else None, len(rules), default_action, binth,
                                 C.byref(words), C.byref(nw), C.byref(st))
    if rc != 0:
        raise ValueError(f"ppe_acl_build_image failed: {rc}")
    img = np.ctypeslib.as_array(words, shape=(nw.value,)).copy()
    lib.ppe_acl_free_image(words)
    return img, st.as_dict()
