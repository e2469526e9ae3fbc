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
    assert lib.ppe_abi_version() == 1


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
    assert C.sizeof(abi.Result) == 56
    assert C.sizeof(abi.Cfg) == 16
    assert C.sizeof(abi.Counters) == 256
