"""Thin Python handle over one ppe_ctx_t (one GPU).  Every call goes through libppe_hip.so."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi


class PPEError(RuntimeError):
    pass


class Engine:
    def __init__(self, device: int = 0, lib=None):
        self.lib = lib or abi.load()
        self.ctx = C.c_void_p()
        rc = self.lib.ppe_ctx_create(int(device), C.byref(self.ctx))
        if rc != 0:
            raise PPEError(f"ppe_ctx_create(device={device}) failed: {rc} (is a GPU visible?)")
        self.device = int(device)

    # ---- lifecycle ----
    def close(self):
        if self.ctx:
            self.lib.ppe_ctx_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc, what):
        if rc != 0:
            err = self.lib.ppe_last_error(self.ctx)
            raise PPEError(f"{what} failed: {rc}: {err.decode() if err else ''}")

    # ---- rules ----
    def commit(self, rules: np.ndarray, used: np.ndarray | None = None,
               default_action: int = abi.ACL_RULE_ACTION_DROP) -> dict:
        rules = np.ascontiguousarray(rules, dtype=abi.RULE_DTYPE)
        if used is not None:
            used = np.ascontiguousarray(used, dtype=np.uint8)
        st = abi.AclStats()
        rc = self.lib.ppe_rules_commit(self.ctx, rules.ctypes.data if len(rules) else None,
                                       used.ctypes.data if used is not None else None, len(rules),
                                       int(default_action), C.byref(st))
        self._check(rc, "ppe_rules_commit")
        return st.as_dict()

    def stage(self, rules: np.ndarray, used: np.ndarray | None = None,
              default_action: int = abi.ACL_RULE_ACTION_DROP) -> tuple[int, dict]:
        """ppe_rules_stage: build and upload the back classifier without publishing it; returns (token, stats)."""
        rules = np.ascontiguousarray(rules, dtype=abi.RULE_DTYPE)
        if used is not None:
            used = np.ascontiguousarray(used, dtype=np.uint8)
        st = abi.AclStats()
        tok = C.c_uint64(0)
        rc = self.lib.ppe_rules_stage(self.ctx, rules.ctypes.data if len(rules) else None,
                                      used.ctypes.data if used is not None else None, len(rules),
                                      int(default_action), C.byref(st), C.byref(tok))
        self._check(rc, "ppe_rules_stage")
        return tok.value, st.as_dict()

    def publish(self, token: int) -> None:
        """ppe_rules_publish: the staged classifier of `token` runs for later launches."""
        self._check(self.lib.ppe_rules_publish(self.ctx, int(token)), "ppe_rules_publish")

    def image(self) -> np.ndarray:
        n = C.c_uint32(0)
        self._check(self.lib.ppe_acl_image(self.ctx, None, C.byref(n)), "ppe_acl_image")
        out = np.zeros(n.value, np.uint32)
        self._check(self.lib.ppe_acl_image(self.ctx, out.ctypes.data, C.byref(n)), "ppe_acl_image")
        return out

    # ---- classify ----
    @staticmethod
    def cfg(unsupport_proto_action=0, syn_check=1, now_seconds=0) -> abi.Cfg:
        return abi.Cfg(int(unsupport_proto_action), int(syn_check), int(now_seconds))

    def classify_ptrs(self, hdr: int, lens: int, n: int, stride: int, out: dict, cfg: abi.Cfg | None = None,
                      ts: int | None = None, stream: int | None = None):
        """Device-pointer form (ppe_classify): enqueue on `stream` (hipStream_t as int) and return."""
        b = abi.Batch(hdr, lens, ts, int(n), int(stride))
        r = abi.Result(out.get("verdict"), out.get("flow_hash"), out.get("acl_hit"), out.get("fw_idx"),
                       out.get("drop_idx"), out.get("tile_cnt"), out.get("tuple"), out.get("part8"), out.get("packed"))
        rc = self.lib.ppe_classify(self.ctx, C.byref(b), C.byref(r), C.byref(cfg or self.cfg()), stream)
        self._check(rc, "ppe_classify")

    def classify_torch(self, hdr, lens, out: dict, cfg: abi.Cfg | None = None, ts=None, stream=None):
        """Tensors on this engine's GPU; `out` maps output names to torch tensors (or None)."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        stride = hdr.shape[1]
        ptrs = {k: (v.data_ptr() if v is not None else None) for k, v in out.items()}
        if ptrs.get("part_idx"):  # partition layout: one list passed as both fw_idx and drop_idx
            ptrs["fw_idx"] = ptrs["drop_idx"] = ptrs.pop("part_idx")
        self.classify_ptrs(hdr.data_ptr(), lens.data_ptr(), lens.numel(), stride, ptrs, cfg,
                           ts.data_ptr() if ts is not None else None, s.cuda_stream)

    def classify_host(self, hdr: np.ndarray, lens: np.ndarray, ts: np.ndarray | None = None,
                      cfg: abi.Cfg | None = None, chunk: int = 0, outputs=("verdict", "flow_hash", "acl_hit"),
                      ) -> dict:
        """Host-buffer form (ppe_classify_host: pipelined H2D → classify → D2H).  hdr: (n, stride) uint8."""
        hdr = np.ascontiguousarray(hdr, dtype=np.uint8)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        n, stride = hdr.shape
        res = {}
        if "verdict" in outputs:
            res["verdict"] = np.zeros(n, np.uint32)
        if "flow_hash" in outputs:
            res["flow_hash"] = np.zeros(n, np.uint32)
        if "acl_hit" in outputs:
            res["acl_hit"] = np.zeros(n, np.int32)
        if "fw_idx" in outputs:
            res["fw_idx"] = np.zeros(n, np.uint32)
        if "drop_idx" in outputs:
            res["drop_idx"] = np.zeros(n, np.uint32)
        if "tile_cnt" in outputs:
            res["tile_cnt"] = np.zeros((n + 63) // 64, np.uint32)
        if "part_idx" in outputs:  # partition layout: one list passed as both fw_idx and drop_idx
            res["part_idx"] = np.zeros(n, np.uint32)
        if "tuple" in outputs:
            res["tuple"] = np.zeros((n, 4), np.uint32)
        if ts is not None:
            ts = np.ascontiguousarray(ts, dtype=np.uint64)
        b = abi.Batch(hdr.ctypes.data, lens.ctypes.data, ts.ctypes.data if ts is not None else None, n, stride)
        g = lambda k: res[k].ctypes.data if k in res else None  # noqa: E731
        fw, dr = (g("part_idx"), g("part_idx")) if "part_idx" in res else (g("fw_idx"), g("drop_idx"))
        r = abi.Result(g("verdict"), g("flow_hash"), g("acl_hit"), fw, dr, g("tile_cnt"), g("tuple"))
        rc = self.lib.ppe_classify_host(self.ctx, C.byref(b), C.byref(r), C.byref(cfg or self.cfg()), int(chunk))
        self._check(rc, "ppe_classify_host")
        return res

    # ---- flow table (ppe_flow_*, dataplane/src/flow/flow.c) ----
    def flow_create(self, capacity: int = 0, max_batch: int = 0):
        self._check(self.lib.ppe_flow_create(self.ctx, int(capacity), int(max_batch)), "ppe_flow_create")

    def flow_destroy(self):
        self._check(self.lib.ppe_flow_destroy(self.ctx), "ppe_flow_destroy")

    def classify_flow_torch(self, hdr, lens, out: dict, cfg: abi.Cfg | None = None, ts=None, stream=None):
        """ppe_classify_flow on tensors of this engine's GPU (same `out` convention as classify_torch)."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        ptrs = {k: (v.data_ptr() if v is not None else None) for k, v in out.items()}
        if ptrs.get("part_idx"):
            ptrs["fw_idx"] = ptrs["drop_idx"] = ptrs.pop("part_idx")
        b = abi.Batch(hdr.data_ptr(), lens.data_ptr(), ts.data_ptr() if ts is not None else None, lens.numel(),
                      hdr.shape[1])
        r = abi.Result(ptrs.get("verdict"), ptrs.get("flow_hash"), ptrs.get("acl_hit"), ptrs.get("fw_idx"),
                       ptrs.get("drop_idx"), ptrs.get("tile_cnt"), ptrs.get("tuple"), ptrs.get("part8"),
                       ptrs.get("packed"))
        self._check(self.lib.ppe_classify_flow(self.ctx, C.byref(b), C.byref(r), C.byref(cfg or self.cfg()),
                                               s.cuda_stream), "ppe_classify_flow")

    def flow_age(self, now: int, timeout: int = 20) -> int:
        d = C.c_uint64(0)
        self._check(self.lib.ppe_flow_age(self.ctx, int(now), int(timeout), C.byref(d)), "ppe_flow_age")
        return d.value

    def flow_info(self) -> dict:
        fi = abi.FlowInfo()
        self._check(self.lib.ppe_flow_info(self.ctx, C.byref(fi)), "ppe_flow_info")
        return fi.as_dict()

    def flow_clear_stat(self):
        self._check(self.lib.ppe_flow_clear_stat(self.ctx), "ppe_flow_clear_stat")

    def flow_dump(self) -> np.ndarray:
        n = C.c_uint32(0)
        self._check(self.lib.ppe_flow_dump(self.ctx, None, 0, C.byref(n)), "ppe_flow_dump")
        out = np.zeros(n.value, abi.FLOW_ENTRY_DTYPE)
        if n.value:
            self._check(self.lib.ppe_flow_dump(self.ctx, out.ctypes.data, n.value, C.byref(n)), "ppe_flow_dump")
        return out

    def acl_lookup_host(self, tuple_: np.ndarray, macs: np.ndarray | None = None, ts: np.ndarray | None = None,
                        now_seconds: int = 0):
        tuple_ = np.ascontiguousarray(tuple_, dtype=np.uint32)
        n = tuple_.shape[0]
        if macs is not None:
            macs = np.ascontiguousarray(macs, dtype=np.uint32)
        if ts is not None:
            ts = np.ascontiguousarray(ts, dtype=np.uint64)
        hit = np.zeros(n, np.int32)
        act = np.zeros(n, np.uint32)
        t = abi.Tuples(tuple_.ctypes.data, macs.ctypes.data if macs is not None else None,
                       ts.ctypes.data if ts is not None else None, n)
        self._check(self.lib.ppe_acl_lookup_host(self.ctx, C.byref(t), hit.ctypes.data, act.ctypes.data,
                                                 int(now_seconds)), "ppe_acl_lookup_host")
        return hit, act

    # ---- counters / timing ----
    def counters(self) -> dict:
        c = abi.Counters()
        self._check(self.lib.ppe_counters_read(self.ctx, C.byref(c)), "ppe_counters_read")
        return c.as_dict()

    def clear_counters(self):
        self._check(self.lib.ppe_counters_clear(self.ctx), "ppe_counters_clear")

    def timing(self, on: bool = True):
        self._check(self.lib.ppe_timing_enable(self.ctx, 1 if on else 0), "ppe_timing_enable")

    def timing_read(self, reset: bool = True):
        ms = C.c_double()
        n = C.c_uint32()
        self._check(self.lib.ppe_timing_read(self.ctx, C.byref(ms), C.byref(n), 1 if reset else 0),
                    "ppe_timing_read")
        return ms.value, n.value

    def tuning(self, **kw) -> dict:
        """Read (and with keyword arguments, set) the launch tuning: block, blocks_per_cu, pipeline, lds_image."""
        t = abi.Tuning()
        self._check(self.lib.ppe_get_tuning(self.ctx, C.byref(t)), "ppe_get_tuning")
        if kw:
            for k, v in kw.items():
                setattr(t, k, int(v))
            self._check(self.lib.ppe_set_tuning(self.ctx, C.byref(t)), "ppe_set_tuning")
        return t.as_dict()

    def launch_info(self) -> dict:
        g, b, l, v = C.c_uint32(), C.c_uint32(), C.c_uint32(), C.c_uint32()
        self._check(self.lib.ppe_launch_info(self.ctx, C.byref(g), C.byref(b), C.byref(l), C.byref(v)),
                    "ppe_launch_info")
        return {"grid": g.value, "block": b.value, "lds_bytes": l.value,
                "image": ("global", "lds", "split")[v.value & 15], "fetch": {0: "none", 1: "hoist", 3: "multi", 5: "cut"}.get(v.value >> 4, f"v{v.value >> 4}")}

    def sync(self):
        self._check(self.lib.ppe_sync(self.ctx), "ppe_sync")


def decode_verdict(v: np.ndarray):
    v = np.asarray(v, dtype=np.uint32)
    return v & 0xFF, (v >> 8) & 0xFF, v >> 16


class Defrag:
    """One device FCB table (ppe_defrag_create) on an Engine's GPU: IPv4 reassembly of the fragments ppe_classify
    PUNTs (dataplane/src/decode/decode-defrag.c).  Every call goes through libppe_hip.so."""

    def __init__(self, engine: Engine, fcb_max=0, cache_max=0, frag_buf_bytes=0, reasm_buf_bytes=0, max_batch=0):
        self.eng = engine
        self.lib = engine.lib
        self.h = C.c_void_p()
        cfg = abi.DefragCfg(fcb_max, cache_max, frag_buf_bytes, reasm_buf_bytes, max_batch, 0)
        rc = self.lib.ppe_defrag_create(engine.ctx, C.byref(cfg), C.byref(self.h))
        if rc != 0:
            raise PPEError(f"ppe_defrag_create failed: {rc}")
        self.info_ = self.info()

    def close(self):
        if self.h:
            self.lib.ppe_defrag_destroy(self.h)
            self.h = C.c_void_p()

    def _check(self, rc, what):
        if rc != 0:
            err = self.lib.ppe_defrag_last_error(self.h)
            raise PPEError(f"{what} failed: {rc}: {err.decode() if err else ''}")

    def alloc_out(self, n: int, hdr_stride: int = 128, full: bool = True):
        """Device output tensors for a batch of n fragments."""
        import torch
        dev = torch.device("cuda", self.eng.device)
        cm = self.info_["cache_max"]
        out = dict(status=torch.empty(n, dtype=torch.int32, device=dev),
                   dgram_of=torch.empty(n, dtype=torch.int32, device=dev),
                   dgram_hdr=torch.empty((n, hdr_stride), dtype=torch.uint8, device=dev),
                   dgram_len=torch.empty(n, dtype=torch.int32, device=dev),
                   dgram_frags=torch.empty((n, cm), dtype=torch.int64, device=dev),
                   n_dgram=torch.zeros(1, dtype=torch.int32, device=dev))
        if full:
            out["dgram_pkt"] = torch.empty((n, self.info_["reasm_buf_bytes"]), dtype=torch.uint8, device=dev)
        return out

    def run_torch(self, pkt, off, lens, out: dict, now: int, ids=None, stream=None):
        """ppe_defrag on tensors of the engine's GPU: pkt (u8 arena), off (i64), lens (i32), ids (i64, optional)."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(self.eng.device)
        n = lens.numel()
        b = abi.FragBatch(pkt.data_ptr(), off.data_ptr(), lens.data_ptr(), ids.data_ptr() if ids is not None else None,
                          n, 0, int(now))
        g = lambda k: out[k].data_ptr() if out.get(k) is not None else None
        o = abi.DefragOut(g("status"), g("dgram_of"), g("dgram_hdr"), g("dgram_len"), g("dgram_pkt"),
                          g("dgram_frags"), g("n_dgram"), out["dgram_hdr"].shape[1], 0)
        self._check(self.lib.ppe_defrag(self.h, C.byref(b), C.byref(o), s.cuda_stream), "ppe_defrag")

    def age(self, now: int, timeout: int = 20):
        """Frag_defrag_timeout: returns (dropped fragment ids, FCBs freed)."""
        cap = self.info_["fcb_max"] * self.info_["cache_max"]
        ids = np.zeros(cap, np.uint64)
        nd, nf = C.c_uint32(0), C.c_uint32(0)
        self._check(self.lib.ppe_defrag_age(self.h, int(now), int(timeout), ids.ctypes.data, cap, C.byref(nd),
                                            C.byref(nf)), "ppe_defrag_age")
        return ids[:min(nd.value, cap)], nf.value

    def info(self) -> dict:
        fi = abi.DefragInfo()
        self._check(self.lib.ppe_defrag_info(self.h, C.byref(fi)), "ppe_defrag_info")
        return fi.as_dict()

