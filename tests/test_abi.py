"""The C-ABI library loads and exports every symbol the include/*.h headers declare (no GPU needed)."""
import ctypes as C
import re
from pathlib import Path

import pytest

from ppe import abi

ROOT = Path(__file__).resolve().parent.parent


def header_functions():
    names = set()
    for h in (ROOT / "include").glob("*.h"):
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        text = re.sub(r"//.*", "", text)
        for m in re.finditer(r"^\s*(?:extern\s+)?[A-Za-z_][\w\s\*]*?\b([A-Za-z_]\w*)\s*\(([^;{]*)\)\s*;", text, re.M):
            name = m.group(1)
            if name in ("typedef", "int", "void") or "(*" in m.group(0):
                continue
            names.add(name)
    return names


def test_library_loads():
    lib = abi.load()
    assert lib.ppe_abi_version() == abi.ABI_VERSION == 8


def test_every_declared_function_is_exported():
    lib = abi.load()
    declared = header_functions()
    assert len(declared) >= 40, declared
    missing = [n for n in sorted(declared) if not hasattr(lib, n)]
    assert not missing, f"declared in include/*.h but not exported: {missing}"
    assert set(abi.EXPORTS) <= declared | set(abi.EXPORTS)
    for n in abi.EXPORTS:
        assert hasattr(lib, n), n


def test_exported_data_symbols():
    lib = abi.load()
    for n in abi.EXPORTED_DATA:
        C.c_int.in_dll(lib, n)


def test_no_device_means_loud_failure():
    """Without a GPU the engine refuses to create a context (there is no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = abi.load()
    ctx = C.c_void_p()
    assert lib.ppe_ctx_create(0, C.byref(ctx)) == -19  # PPE_ENODEV
    assert not ctx


def test_struct_layouts():
    assert abi.RULE_DTYPE.itemsize == 60  # include/rpc-common.h:97-114, packed
    assert C.sizeof(abi.Batch) == 32
    assert C.sizeof(abi.Result) == 72  # part8 (ABI version 4), packed (8)
    assert C.sizeof(abi.Cfg) == 16
    assert C.sizeof(abi.Tuning) == 20  # batches_per_launch (ABI version 2)
    assert C.sizeof(abi.Counters) == 256
    assert C.sizeof(abi.AclStats) == 56  # cut_bits / cut_entries (ABI version 6)


# LP64 offsets of the reference's mbuf_t (dataplane/src/include/mbuf.h:23-87, with cvmx_buf_ptr_t a 64-bit word and
# TCPVars {TCPOpt[1]; TCPOpt *} = 24 B, decode-tcp.h:24-46), derived by hand from the declaration order; the
# reference's own memset of the struct is 232 B (oct-rxtx.c:190-192)
REF_MBUF_OFFSETS = dict(
    magic_flag=0, pkt_space=4, flow_log=5, frag_len=6, packet_ptr=8, next=16, pkt_ptr=24, ethh=32, vlanh=40,
    network_header=48, transport_header=56, input_port=64, eth_dst=68, eth_src=74, ipv4=80, sport=88, dport=90,
    proto=92, vlan_idx=93, payload_len=94, vlan_id=96, defrag_id=98, timestamp=104, payload=112, tcpvars=120,
    frag_offset=144, tcp_reasm_overlap=146, pkt_totallen=148, flags=152, fcb_hash=156, fcb=160, fragments=168,
    flow=176, tcp_seg_raw=184, tcp_seg_raw_tail=192, tcp_seg_reassem=200, alState=208, FreeState=216, tag=224)


def test_mbuf_layout_matches_reference(tmp_path):
    """include/ppe_decode.h's mbuf_t keeps every reference field at its reference offset (compiled with gcc), and the
    ctypes mirror (ppe.abi.Mbuf) agrees with the compiler."""
    import subprocess
    names = list(REF_MBUF_OFFSETS) + ["ppe_verdict", "ppe_flow_hash", "ppe_acl_hit", "user"]
    src = tmp_path / "off.c"
    src.write_text("#include <stdio.h>\n#include <stddef.h>\n#include \"ppe_decode.h\"\nint main(void){\n" +
                   "".join(f'printf("{n} %zu\\n", offsetof(mbuf_t, {n}));\n' for n in names) +
                   'printf("sizeof %zu\\n", sizeof(mbuf_t));\n'
                   'mbuf_t m; m.tcpvars.ws = 0; (void)m;\nreturn 0;}\n')
    exe = tmp_path / "off"
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", f"-I{ROOT / 'include'}", str(src), "-o", str(exe)],
                   check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], check=True, capture_output=True,
                                                       text=True).stdout.splitlines())
    got = {k: int(v) for k, v in got.items()}
    for k, off in REF_MBUF_OFFSETS.items():
        assert got[k] == off, (k, got[k], off)
    assert got["ppe_verdict"] >= 228
    ct = {f[0]: getattr(abi.Mbuf, f[0]).offset for f in abi.Mbuf._fields_}
    ct["ipv4"] = ct["sip"]
    for k in names:
        assert ct[k] == got[k], k
    assert C.sizeof(abi.Mbuf) == got["sizeof"]


def test_running_tree_switch_links(tmp_path):
    """dp_cmd.c's get_back_acltree / set_running_acltree (dp_cmd.c:1963-1985), written against include/ppe_acl.h and
    its rwlock stand-in, compile and link against the library and switch the exported running pointer (no GPU
    call: the engine context is never created)."""
    import subprocess
    src = tmp_path / "sw.c"
    src.write_text(
        '#include "ppe_acl.h"\n'
        "static unit_tree_t *back_tree(void) {\n"
        "    return g_acltree_running == (unsigned long)(void *)&g_acltree_1 ? &g_acltree_2 : &g_acltree_1;\n"
        "}\n"
        "static void set_running(unit_tree_t *t) {\n"
        "    write_lock(&acltree_running_rwlock);\n"
        "    g_acltree_running = (unsigned long)(void *)t;\n"
        "    write_unlock(&acltree_running_rwlock);\n"
        "}\n"
        "int main(void) {\n"
        "    unit_tree_t *a = back_tree();\n"
        "    set_running(a);\n"
        "    unit_tree_t *b = back_tree();\n"
        "    read_lock(&acltree_running_rwlock);\n"
        "    const int ok = a == &g_acltree_1 && b == &g_acltree_2 && read_trylock(&acltree_running_rwlock) &&\n"
        "                   !write_trylock(&acltree_running_rwlock);\n"
        "    read_unlock(&acltree_running_rwlock);\n"
        "    read_unlock(&acltree_running_rwlock);\n"
        "    return ok && write_trylock(&acltree_running_rwlock) ? 0 : 1;\n"
        "}\n")
    exe = tmp_path / "sw"
    lib = ROOT / "packet-process-engine_amd"
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", f"-I{ROOT / 'include'}", str(src), f"-L{lib}", "-lppe_hip",
                    f"-Wl,-rpath,{lib}", "-o", str(exe)], check=True)
    assert subprocess.run([str(exe)]).returncode == 0
