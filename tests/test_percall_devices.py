"""CPU: device selection of the per-call drop-in path (include/ecamd_host.h
ecamd_percall_device_plan).  liberasurecode_encode / _decode / _reconstruct_fragment are called
concurrently from many threads under a shared read lock (src/erasurecode.c:414, 543, 769); on an
8-GPU node the calls go round-robin over every visible device (or the ECAMD_PERCALL_DEVICES
subset), each device with its own staging pool, so the drop-in uses all PCIe links."""
import ctypes as C

import pytest

from liberasurecode_amd import _lib


def plan(ndev, spec, cap=16):
    h = _lib.host()
    f = h.ecamd_percall_device_plan
    f.restype = C.c_int
    f.argtypes = [C.c_int, C.c_char_p, C.POINTER(C.c_int), C.c_int]
    out = (C.c_int * cap)(*([-1] * cap))
    n = f(ndev, None if spec is None else spec.encode(), out, cap)
    return list(out[:n])


@pytest.mark.parametrize("ndev", [1, 2, 8])
def test_default_is_every_device(ndev):
    assert plan(ndev, None) == list(range(ndev))
    assert plan(ndev, "") == list(range(ndev))


def test_subset_spec():
    assert plan(8, "2,5") == [2, 5]
    assert plan(8, " 7 , 0 ") == [7, 0]
    assert plan(8, "3,3,1,3") == [3, 1]          # repeats dropped
    assert plan(8, "9,1,-1") == [1]              # out of range dropped ("-1" parses as -1)
    assert plan(8, "12") == list(range(8))       # names none of the devices: all
    assert plan(4, "x") == list(range(4))


def test_capacity_and_no_device():
    assert plan(8, None, cap=3) == [0, 1, 2]
    assert plan(0, None) == []


def test_round_robin_balance():
    devs = plan(8, None)
    calls = [devs[n % len(devs)] for n in range(80)]
    assert all(calls.count(d) == 10 for d in devs)


def test_current_spec_plans_every_device():
    """ECAMD_PERCALL_DEVICES=current: the plan keeps every device (the pool may serve any of
    them) and each call runs on the caller's current device (hostio.cpp pick_device) -- what
    liberasurecode_amd/shard.py sets for its one-process-per-GPU ranks."""
    assert plan(8, "current") == list(range(8))

