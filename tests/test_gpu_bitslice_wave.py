"""GPU: the bitsliced kernel in one-wave 4 KiB tiles for every map width it takes (host/bitslice.cpp,
hip/ecamd_device.hip launch_bitslice), against the CPU oracle, bit-exact, with the launch counter
proving the bitsliced kernel ran:

* 1-2-output maps (knob bs_narrow_min_k): single-destination reconstruct of a data and a parity
  fragment (liberasurecode_rs_vand_reconstruct, src/builtin/rs_vand/liberasurecode_rs_vand.c:483-558;
  the call Swift's reconstructor makes, src/erasurecode.c:748-949), decodes of 1 and 2 lost
  fragments (:426-481), C2's 2-parity encode (:399-410);
* the inputs straight into registers (bs_wave_depth 0) or through the one-wave LDS-DMA ring, 2 and 4
  inputs deep (bs_wave_depth 2 / 4), with one workgroup per tile (bs_grid 1) and grid-stride
  workgroups that carry the ring across tiles (bs_grid 0);
* fragments whose last 4 KiB tile is partial (the tail runs on the LDS-table kernel)."""
import ctypes

import numpy as np
import pytest

import oracle_lib as orc
from ecdata import stripe_fragments
from liberasurecode_amd import _lib
from liberasurecode_amd import device as D

pytestmark = pytest.mark.gpu

KNOBS = {"bitslice": 1, "bs_wave_depth": 0, "bs_narrow_min_k": -1, "bs_grid": 1}


@pytest.fixture(params=[(0, 1), (2, 1), (4, 1), (2, 0)], ids=["regs", "ring2", "ring4", "ring2_gridstride"])
def form(request):
    d = _lib.dev()
    depth, grid = request.param
    d.ecamd_tune(b"bitslice", 2)  # wait for each compile: every launch takes the bitsliced kernel
    d.ecamd_tune(b"bs_wave_depth", depth)
    d.ecamd_tune(b"bs_grid", grid)
    d.ecamd_tune(b"bs_narrow_min_k", 1)  # 1-2-output maps too, whatever k
    d.ecamd_tune(b"small_chunks", 0)  # small batches would otherwise take the small-launch kernel
    yield d
    d.ecamd_tune(b"small_chunks", -1)
    for k, v in KNOBS.items():
        d.ecamd_tune(k.encode(), v)


def _launches():
    f = _lib.dev().ecamd_bitslice_launches
    f.restype = ctypes.c_longlong
    return f()


def _batch(k, m, bs, S, seed):
    lay = D.Layout.alloc(k + m, bs, S)
    lay.fill_splitmix(nfrags=k, stripe0=seed)
    want = np.stack([np.concatenate([stripe_fragments(seed + s, k, bs),
                                     orc.encode(k, m, stripe_fragments(seed + s, k, bs))])
                     for s in range(S)])
    return lay, want


@pytest.mark.parametrize("k,m,bs,S", [(10, 4, 4096 * 5 + 100, 5), (4, 2, 65536, 6), (10, 2, 4096 * 3, 40),
                                      (20, 1, 4096 * 2 + 2, 3)])
def test_encode_exact(form, k, m, bs, S):
    lay, want = _batch(k, m, bs, S, 7)
    n0 = _launches()
    D.rs_encode(k, m, lay)
    assert (lay.download_stripes() == want).all()
    assert _launches() > n0
    lay.buf.free()


@pytest.mark.parametrize("k,m,lost", [(10, 4, [3]), (10, 4, [12]), (10, 4, [0, 11]), (10, 4, [5, 6]),
                                      (10, 4, [0, 5, 10, 13]), (20, 8, [7]), (20, 8, [0, 27]),
                                      (4, 2, [0, 4])])
def test_decode_exact(form, k, m, lost):
    bs, S = 4096 * 4 + 48, 6
    lay, want = _batch(k, m, bs, S, 19)
    host = want.copy()
    host[:, lost] = 0x5A  # garbage in the lost slots
    lay.upload_stripes(host)
    n0 = _launches()
    D.rs_decode(k, m, lost, lay)
    assert (lay.download_stripes() == want).all()
    assert _launches() > n0
    lay.buf.free()


@pytest.mark.parametrize("k,m,missing,dest", [(10, 4, [3], 3), (10, 4, [12], 12), (10, 4, [0, 5, 10, 13], 13),
                                              (10, 4, [0, 5, 10, 13], 5), (20, 8, list(range(8)), 5),
                                              (20, 8, [0, 2, 4, 6, 20, 22, 24, 26], 22)])
def test_reconstruct_exact(form, k, m, missing, dest):
    bs, S = 4096 * 8 + 2, 5
    lay, want = _batch(k, m, bs, S, 23)
    host = want.copy()
    host[:, missing] = 0xC3
    lay.upload_stripes(host)
    n0 = _launches()
    D.rs_reconstruct(k, m, missing, dest, lay)
    got = lay.download_stripes()
    assert (got[:, dest] == want[:, dest]).all()
    others = [f for f in range(k + m) if f != dest]
    assert (got[:, others] == host[:, others]).all()  # nothing else written
    assert _launches() > n0
    lay.buf.free()


def test_narrow_knob_off_keeps_tables():
    """bs_narrow_min_k 0: 1-2-output maps stay on the LDS-table kernel (no bitsliced launch), same bytes."""
    d = _lib.dev()
    k, m = 10, 4
    lay, want = _batch(k, m, 4096 * 4, 3, 29)
    try:
        d.ecamd_tune(b"bitslice", 2)
        d.ecamd_tune(b"bs_narrow_min_k", 0)
        host = want.copy()
        host[:, [3]] = 0
        lay.upload_stripes(host)
        n0 = _launches()
        D.rs_reconstruct(k, m, [3], 3, lay)
        assert (lay.download_stripes() == want).all()
        assert _launches() == n0
    finally:
        for key, v in KNOBS.items():
            d.ecamd_tune(key.encode(), v)
        lay.buf.free()


@pytest.mark.parametrize("streams", [1, 4])
def test_decode_multi_patterns_bitsliced(streams):
    """ecamd_rs_decode_multi over a heterogeneous (10, 4) batch -- the four patterns tools/multi_bench.py
    times plus ones no build ships ({1,2,3,4}, {5,9,11}) and single / 2-loss ones -- every group on the
    bitsliced kernel (knob bitslice 2 compiles what is not shipped), stripe lists in the default
    one-wave form, byte-exact against the oracle's decode of each stripe; knob multi_streams 4 spreads
    the per-pattern launches over the caller's stream and 3 forked pool streams."""
    d = _lib.dev()
    d.ecamd_tune(b"bitslice", 2)
    d.ecamd_tune(b"multi_streams", streams)
    d.ecamd_tune(b"small_chunks", 0)
    try:
        k, m, bs, S = 10, 4, 4096 * 3, 48
        pats = [[0, 1, 2, 3], [4, 5, 6, 7], [0, 5, 10, 13], [2, 3, 8, 9], [1, 2, 3, 4], [6], [2, 7], [5, 9, 11]]
        per = [pats[s % len(pats)] for s in range(S)]
        lay, want = _batch(k, m, bs, S, 41)
        host = want.copy()
        for s, p in enumerate(per):
            host[s, p] = 0xC3
        lay.upload_stripes(host)
        n0 = _launches()
        D.rs_decode_multi(k, m, per, lay)
        assert _launches() - n0 >= len(pats)
        assert (lay.download_stripes() == want).all()
        lay.buf.free()
    finally:
        d.ecamd_tune(b"multi_streams", 1)
        d.ecamd_tune(b"small_chunks", -1)
        d.ecamd_tune(b"bitslice", 1)
