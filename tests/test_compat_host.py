"""Decode() burst bookkeeping of the PPE compat layer (include/ppe_decode.h) on the host, without a GPU: with no
engine context every flush fails with PPE_ENODEV, and the reference's contract still holds — every queued mbuf ends
in the drop hook (output_drop_proc, dataplane/src/decode/decode.c:24-27), none is lost or delivered twice — while the
burst size is changed under traffic (a raised cap must grow the burst array, not overrun it)."""
import ctypes as C
import threading

import pytest

from ppe import abi

HOOK = C.CFUNCTYPE(None, C.POINTER(abi.Mbuf))


@pytest.fixture()
def lib():
    import torch
    if torch.cuda.is_available():
        pytest.skip("host-only bookkeeping test (a GPU would classify the bursts)")
    lib = abi.load()
    lib.DP_Acl_Rule_Release()  # no context: flushes fail with PPE_ENODEV
    lib.ppe_set_output_hooks.argtypes = [HOOK, HOOK, HOOK]
    yield lib
    lib.ppe_set_output_hooks(HOOK(), HOOK(), HOOK())
    lib.Decode_Set_Burst(4096)


def install(lib, got, reenter=None):
    def mk(key):
        def f(m):
            got.setdefault(key, []).append(C.addressof(m.contents))
            if reenter is not None and key == "drop":
                reenter(m)
        return HOOK(f)
    hooks = (mk("fw"), mk("drop"), mk("punt"))
    lib.ppe_set_output_hooks(*hooks)
    return hooks


def test_raise_cap_after_traffic_started(lib):
    got = {}
    hooks = install(lib, got)  # noqa: F841 (keep the callbacks alive)
    mb = (abi.Mbuf * 20)()
    lib.Decode_Set_Burst(4)
    for i in range(3):
        lib.Decode(C.byref(mb[i]))
    assert got == {}  # 3 < 4 queued
    lib.Decode_Set_Burst(8)  # raised with 3 queued: the array must grow to 8 before the 4th..8th append
    for i in range(3, 8):
        lib.Decode(C.byref(mb[i]))
    assert len(got["drop"]) == 8  # the 8th flushed the burst; no context, so all 8 dropped
    lib.Decode_Set_Burst(2)  # lowered below what is queued
    for i in range(8, 11):
        lib.Decode(C.byref(mb[i]))
    assert lib.Decode_Flush() in (0, -19)
    base = C.addressof(mb)
    idx = sorted((a - base) // C.sizeof(abi.Mbuf) for a in got["drop"])
    assert idx == list(range(11)) and "fw" not in got and "punt" not in got


def test_failed_flush_drops_everything_and_reports(lib):
    got = {}
    hooks = install(lib, got)  # noqa: F841
    mb = (abi.Mbuf * 5)()
    lib.Decode_Set_Burst(100)
    for i in range(5):
        lib.Decode(C.byref(mb[i]))
    assert lib.Decode_Flush() == -19  # PPE_ENODEV
    assert len(got["drop"]) == 5
    assert lib.Decode_Flush() == 0  # nothing left queued


def test_hook_may_reenter_decode(lib):
    """The hooks run with no lock held: a drop hook that feeds packets back into Decode() does not deadlock."""
    got = {}
    extra = (abi.Mbuf * 4)()
    fed = []

    def reenter(m):
        if len(fed) < 4:
            fed.append(1)
            lib.Decode(C.byref(extra[len(fed) - 1]))

    hooks = install(lib, got, reenter)  # noqa: F841
    mb = (abi.Mbuf * 2)()
    lib.Decode_Set_Burst(1000)
    done = threading.Event()

    def run():  # on its own thread, so a deadlock fails the test instead of hanging it
        for i in range(2):
            lib.Decode(C.byref(mb[i]))
        while lib.Decode_Flush() != 0:
            pass
        done.set()
    t = threading.Thread(target=run)
    t.start()
    t.join(10)
    assert done.is_set(), "Decode_Flush deadlocked on a re-entrant hook"
    assert len(got["drop"]) == 6


def test_bursts_are_per_thread(lib):
    """Each thread flushes only its own burst (the reference decodes on the receiving core)."""
    got = {}
    hooks = install(lib, got)  # noqa: F841
    mb = (abi.Mbuf * 6)()
    lib.Decode_Set_Burst(100)
    for i in range(3):
        lib.Decode(C.byref(mb[i]))
    res = []

    def other():
        for i in range(3, 6):
            lib.Decode(C.byref(mb[i]))
        res.append(lib.Decode_Flush())
    t = threading.Thread(target=other)
    t.start()
    t.join(10)
    assert res == [-19] and len(got["drop"]) == 3
    base = C.addressof(mb)
    assert sorted((a - base) // C.sizeof(abi.Mbuf) for a in got["drop"]) == [3, 4, 5]
    assert lib.Decode_Flush() == -19 and len(got["drop"]) == 6


def test_allocation_failures_still_reach_the_drop_hook(lib):
    """an allocation failure anywhere on the Decode path must not lose an mbuf.  With the test hook
    ppe_compat_debug_fail_alloc(k) the next k allocations fail: a flush whose classify buffers cannot be allocated
    returns PPE_ENOMEM and hands every queued mbuf to the drop hook; a Decode() whose burst cannot grow drops that
    one packet at once; afterwards the path works again."""
    lib.ppe_compat_debug_fail_alloc.argtypes = [C.c_uint32]
    got = {}
    hooks = install(lib, got)  # noqa: F841
    mb = (abi.Mbuf * 12)()
    base = C.addressof(mb)
    idx = lambda key: sorted((a - base) // C.sizeof(abi.Mbuf) for a in got.get(key, []))  # noqa: E731
    lib.Decode_Set_Burst(100)
    for i in range(5):
        lib.Decode(C.byref(mb[i]))
    lib.ppe_compat_debug_fail_alloc(1)  # the flush's first buffer
    assert lib.Decode_Flush() == -12  # PPE_ENOMEM
    assert idx("drop") == [0, 1, 2, 3, 4]
    assert lib.Decode_Flush() == 0  # nothing left queued
    # the burst array was handed back to the burst; a fresh thread's first Decode must allocate it
    res = []

    def fresh():
        lib.ppe_compat_debug_fail_alloc(1)
        lib.Decode(C.byref(mb[5]))  # the burst cannot grow: dropped at once
        res.append(idx("drop"))
        lib.Decode(C.byref(mb[6]))
        res.append(lib.Decode_Flush())  # no context: PPE_ENODEV, mb[6] dropped
    t = threading.Thread(target=fresh)
    t.start()
    t.join(10)
    assert res[0] == [0, 1, 2, 3, 4, 5] and res[1] == -19
    assert idx("drop") == list(range(7)) and "fw" not in got and "punt" not in got
    lib.ppe_compat_debug_fail_alloc(0)


def test_thread_exit_flushes_its_burst(lib):
    """A thread that exits with mbufs queued delivers them (the burst's TLS destructor), exactly once."""
    got = {}
    hooks = install(lib, got)  # noqa: F841
    mb = (abi.Mbuf * 3)()
    lib.Decode_Set_Burst(100)

    def worker():
        for i in range(3):
            lib.Decode(C.byref(mb[i]))
    t = threading.Thread(target=worker)
    t.start()
    t.join(10)
    # (Python's join returns when the thread's interpreter state is gone; the TLS destructors run just after)
    import time
    for _ in range(200):
        if len(got.get("drop", [])) >= 3:
            break
        time.sleep(0.01)
    base = C.addressof(mb)
    assert sorted((a - base) // C.sizeof(abi.Mbuf) for a in got["drop"]) == [0, 1, 2]
