"""GPU: device-level behaviour of libecamd beyond single-launch parity.

* Fragment placement across GPUs (reference anchor: the rs_vand shim's
  fragments_needed, src/backends/rs_vand/liberasurecode_rs_vand.c:119-145): fragment f of every
  stripe goes to device f % device_count() -- over xGMI where that is a peer, a local copy on a
  one-GPU box -- and every destination byte is checked.
* The prepared-map cache is bounded: a long-lived process that meets many distinct erasure
  patterns keeps at most the cache limit of coefficient tables on the device, and evicted maps are
  rebuilt transparently (results stay bit-exact).
* The per-call path restores the caller's current device.
"""
import ctypes as C
import itertools

import numpy as np
import pytest
import torch

import oracle_lib as orc
from ecdata import stripe_fragments
from liberasurecode_amd import _lib
from liberasurecode_amd import device as D

pytestmark = pytest.mark.gpu


def _scatter():
    f = _lib.dev().ecamd_scatter_fragments
    f.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_void_p,
                  C.c_void_p, C.c_void_p, C.c_void_p]
    return f


@pytest.mark.parametrize("lanes", [0, 1, 2])
def test_scatter_fragments_round_robin_devices(lanes):
    """lanes: copy lanes for peer destinations (0, default), for every destination (1: the
    fork / join on one-GPU boxes too), none (2: everything on the caller's stream)."""
    ndev = torch.cuda.device_count()
    k, m, bs, S = 10, 4, 65536 + 48, 5
    lay = D.Layout.alloc(k + m, bs, S)
    stream = D.Stream()
    lay.fill_splitmix(stream=stream)
    D.rs_encode(k, m, lay, stream=stream)
    stream.synchronize()
    src = lay.download_stripes()
    devs = [f % ndev for f in range(k + m)]
    strides = [bs + 16 * (f + 1) for f in range(k + m)]
    bufs = []
    for f in range(k + m):
        torch.cuda.set_device(devs[f])
        bufs.append(D.DeviceBuffer(S * strides[f]))
        bufs[-1].zero()
    torch.cuda.set_device(0)
    h = _lib.dev()
    assert h.ecamd_tune(b"scatter_lanes", lanes) == 0
    try:
        # re-encode right before the scatter on the same stream: the lanes must wait for it
        D.rs_encode(k, m, lay, stream=stream)
        rc = _scatter()(lay.buf.ptr, lay.stripe_stride, lay.frag_stride, bs, k + m, S,
                        _lib.ints(devs), (C.c_void_p * (k + m))(*[b.ptr for b in bufs]),
                        _lib.i64s(strides), stream.handle)
        assert rc == 0, h.ecamd_last_error()
        stream.synchronize()  # the join: the caller's stream covers every lane's copies
    finally:
        h.ecamd_tune(b"scatter_lanes", 0)
    # no device-wide synchronize here: the lanes are non-blocking streams, so only the join into
    # `stream` orders them before these reads
    for f in range(k + m):
        torch.cuda.set_device(devs[f])
        got = bufs[f].download(S * strides[f]).reshape(S, strides[f])[:, :bs]
        assert (got == src[:, f]).all(), f"fragment {f} on device {devs[f]}"
    torch.cuda.set_device(0)
    for f, b in enumerate(bufs):
        torch.cuda.set_device(devs[f])
        b.free()
    torch.cuda.set_device(0)


def test_scatter_reports_the_failing_destination():
    ndev = torch.cuda.device_count()
    lay = D.Layout.alloc(3, 4096, 2)
    dst = D.DeviceBuffer(3 * 4096 * 2)
    rc = _scatter()(lay.buf.ptr, lay.stripe_stride, lay.frag_stride, 4096, 3, 2,
                    _lib.ints([0, ndev + 3, 0]),
                    (C.c_void_p * 3)(dst.ptr, dst.ptr, dst.ptr), _lib.i64s([8192] * 3), None)
    assert rc != 0
    msg = _lib.dev().ecamd_last_error().decode()
    assert "fragment 1" in msg and str(ndev + 3) in msg


def _stats():
    f = _lib.dev().ecamd_map_cache_stats
    f.argtypes = [C.POINTER(C.c_int64)] * 3
    e, b, lim = C.c_int64(), C.c_int64(), C.c_int64()
    assert f(C.byref(e), C.byref(b), C.byref(lim)) == 0
    return e.value, b.value, lim.value


def test_map_cache_is_bounded_and_evictions_stay_exact():
    k, m, bs, S = 20, 8, 256, 2
    lay = D.Layout.alloc(k + m, bs, S)
    lay.fill_splitmix(nfrags=k)
    D.rs_encode(k, m, lay)
    want = lay.download_stripes()
    pats = list(itertools.islice(itertools.combinations(range(k + m), 8), 0, 100000, 97))
    assert len(pats) > 600  # > 100 MiB of tables if nothing were evicted
    peak = 0
    for i, pat in enumerate(pats):
        D.rs_decode(k, m, list(pat), lay)  # 8 outputs: ~180 KiB of tables per pattern
        if i % 50 == 0:
            D.synchronize()
            _, b, lim = _stats()
            peak = max(peak, b)
            assert b <= lim
    entries, b, lim = _stats()
    assert b <= lim and entries < len(pats)
    assert (lay.download_stripes() == want).all()  # every decode on consistent stripes
    # an early pattern was evicted; running it again rebuilds its map and stays bit-exact
    host = want.copy()
    host[:, list(pats[0])] = 0
    lay.upload_stripes(host)
    D.rs_decode(k, m, list(pats[0]), lay)
    assert (lay.download_stripes() == want).all()
    assert peak <= lim


def test_percall_restores_callers_device():
    ndev = torch.cuda.device_count()
    h = _lib.dev()
    k, m, bs = 4, 2, 8192
    data = stripe_fragments(5, k, bs)
    parity = [np.zeros(bs, np.uint8) for _ in range(m)]
    G = orc.generator(k, m)
    coeff = _lib.ints(G[k * k:])
    ins = (C.c_void_p * k)(*[x.ctypes.data for x in data])
    outs = (C.c_void_p * m)(*[x.ctypes.data for x in parity])
    for cur in range(ndev):
        torch.cuda.set_device(cur)
        for _ in range(ndev + 1):  # round-robin touches every device
            assert h.ecamd_host_map_apply(coeff, m, k, ins, outs, bs) == 0
            assert torch.cuda.current_device() == cur
            d = C.c_int(-1)
            h.ecamd_get_device.argtypes = [C.POINTER(C.c_int)]
            assert h.ecamd_get_device(C.byref(d)) == 0 and d.value == cur
    torch.cuda.set_device(0)
    want = orc.encode(k, m, data)
    assert all((parity[i] == want[i]).all() for i in range(m))
