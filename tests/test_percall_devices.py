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
    """ECAMD_PERCALL_DEVICES=current is not a list of ids: the id parser keeps every device;
    hostio.cpp resolves "current" itself, once, to the device current when the plan is built."""
    assert plan(8, "current") == list(range(8))


def test_rank_spec_pins_one_device():
    """shard.py pins each rank's per-call path to its own GPU with an explicit index (a worker
    thread of the rank that never selected a device must not fall back to device 0)."""
    from liberasurecode_amd.shard import percall_devices_spec
    for dev in range(8):
        spec = percall_devices_spec(dev)
        assert plan(8, spec) == [dev]
        calls = [plan(8, spec)[n % 1] for n in range(16)]
        assert set(calls) == {dev}
    import pytest
    with pytest.raises(ValueError):
        percall_devices_spec(-1)

