"""GPU: run-time compiled bitsliced kernels for 8-output passes (hip/ecamd_jit.hip,
host/bitslice.cpp) against the CPU oracle, bit-exact.

Covers encode (C5 shape: liberasurecode_rs_vand_encode, src/builtin/rs_vand/liberasurecode_rs_vand.c:399-410),
decode / reconstruct of 5..8 lost fragments (:426-481, :483-558) -- also k > 20, where the
LDS-table passes split rows and columns but the bitsliced kernel takes all k inputs of each group of
8 outputs, and more than 8 outputs (the rows past 8 stay on the tables) --, fragments with a tail that is
not a whole 16 KiB tile (the tail runs through the LDS-table kernel), heterogeneous batches over
stripe lists, and the knob that turns the bitsliced form off (same bytes).  Every test runs with
the inputs loaded straight into registers (bitslice_depth 0) and through the per-wave LDS-DMA ring
(2 inputs deep; the 4-deep ring in test_ring4_many_tiles); batches with many more tiles than
workgroups exercise the ring's prefetch across tile boundaries and its drain after the last tile."""
import numpy as np
import pytest

import oracle_lib as orc
from ecdata import stripe_fragments
from liberasurecode_amd import _lib
from liberasurecode_amd import device as D

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=[0, 2], ids=["regs", "ring2"])
def sync_compile(request):
    d = _lib.dev()
    d.ecamd_tune(b"bitslice", 2)  # wait for the compile: every launch below takes the JIT kernel
    d.ecamd_tune(b"bitslice_depth", request.param)
    d.ecamd_tune(b"small_chunks", 0)  # small batches would otherwise take the small-launch kernel
    yield d
    d.ecamd_tune(b"bitslice", 1)
    d.ecamd_tune(b"bitslice_depth", DEFAULT_DEPTH)
    d.ecamd_tune(b"small_chunks", -1)


DEFAULT_DEPTH = 0


def test_hiprtc_available():
    assert _lib.dev().ecamd_bitslice_available() == 1


def _batch(k, m, bs, S, seed=3):
    lay = D.Layout.alloc(k + m, bs, S)
    lay.fill_splitmix(nfrags=k, stripe0=seed)
    want = np.stack([np.concatenate([stripe_fragments(seed + s, k, bs),
                                     orc.encode(k, m, stripe_fragments(seed + s, k, bs))])
                     for s in range(S)])
    return lay, want


@pytest.mark.parametrize("k,m,bs", [(20, 8, 65536), (20, 8, 65536 + 4096 + 48), (10, 6, 16384 * 3),
                                    (12, 5, 16384 + 2), (32, 8, 32768), (24, 8, 65536 + 16384 + 6),
                                    (6, 10, 32768), (25, 13, 49152)])
def test_encode_exact(k, m, bs):
    lay, want = _batch(k, m, bs, 3)
    D.rs_encode(k, m, lay)
    assert (lay.download_stripes() == want).all()
    assert _lib.dev().ecamd_bitslice_wait() == 0


@pytest.mark.parametrize("k,m,lost", [(20, 8, list(range(8))), (20, 8, [0, 2, 4, 6, 20, 22, 24, 26]),
                                      (20, 8, [1, 3, 5, 7, 9]), (10, 6, [0, 1, 2, 3, 4, 5]),
                                      (16, 7, [15, 14, 13, 16, 18, 20, 22]),
                                      (24, 8, [0, 1, 2, 3, 4, 5, 6, 7]), (10, 12, list(range(10))),
                                      (32, 8, [1, 3, 5, 7, 32, 34, 36, 38])])
def test_decode_exact(k, m, lost):
    bs = 49152 + 80
    lay, want = _batch(k, m, bs, 4)
    host = want.copy()
    host[:, lost] = 0x5A  # garbage in the lost slots
    lay.upload_stripes(host)
    D.rs_decode(k, m, lost, lay)
    assert (lay.download_stripes() == want).all()


def test_reconstruct_and_multi_exact():
    k, m, bs, S = 20, 8, 32768, 6
    lay, want = _batch(k, m, bs, S, seed=9)
    pats = [list(range(8)), [0, 2, 4, 6, 20, 22, 24, 26], list(range(8)), [3, 4, 5, 6, 7, 21, 22, 23],
            [0, 2, 4, 6, 20, 22, 24, 26], list(range(8))]
    host = want.copy()
    for s, p in enumerate(pats):
        host[s, p] = 0xA5
    lay.upload_stripes(host)
    D.rs_decode_multi(k, m, pats, lay)
    assert (lay.download_stripes() == want).all()
    # single-destination reconstruct stays on the LDS path (1 output) and agrees
    lost8 = want.copy()
    lost8[:, :8] = 0x3C
    lay.upload_stripes(lost8)
    D.rs_reconstruct(k, m, list(range(8)), 5, lay)
    assert (lay.download_stripes()[:, 5] == want[:, 5]).all()


def test_knob_off_gives_the_same_bytes(sync_compile):
    k, m, bs = 20, 8, 65536
    lay, want = _batch(k, m, bs, 2)
    sync_compile.ecamd_tune(b"bitslice", 0)
    D.rs_encode(k, m, lay)
    a = lay.download_stripes()
    sync_compile.ecamd_tune(b"bitslice", 2)
    lay.upload_stripes(np.zeros_like(a))
    lay.fill_splitmix(nfrags=k, stripe0=3)
    D.rs_encode(k, m, lay)
    assert (a == want).all() and (lay.download_stripes() == want).all()


@pytest.mark.parametrize("bs_tps", [16, 1])
@pytest.mark.parametrize("k,m,lost", [(20, 8, None), (20, 8, [0, 2, 4, 6, 20, 22, 24, 26]), (3, 5, None),
                                      (1, 8, None)])
def test_many_tiles_per_workgroup(sync_compile, k, m, lost, bs_tps):
    """ntiles >> workgroups (2 per CU): the same bytes as the LDS-table kernels, which the tests
    above pin to the oracle.  k = 1 and 3 take the shallower ring (prefetch stays within one tile
    ahead).  bs_tps 1: the pass split into launches of one tile per workgroup (6 here)."""
    sync_compile.ecamd_tune(b"bs_tiles_per_slot", bs_tps)
    try:
        _many_tiles(sync_compile, k, m, lost)
    finally:
        sync_compile.ecamd_tune(b"bs_tiles_per_slot", 16)


def _many_tiles(sync_compile, k, m, lost):
    bs, S = 1 << 20, 48
    lay = D.Layout.alloc(k + m, bs, S)
    lay.fill_splitmix(nfrags=k if lost is None else k + m, stripe0=11)
    if lost is not None:
        sync_compile.ecamd_tune(b"bitslice", 0)
        D.rs_encode(k, m, lay)
    ref = None
    for mode in (0, 2):
        sync_compile.ecamd_tune(b"bitslice", mode)
        if lost is None:
            D.rs_encode(k, m, lay)
        else:
            D.rs_decode(k, m, lost, lay)
        got = lay.download_stripes()
        if ref is None:
            ref = got
            host = got.copy()  # the next pass must rewrite these slots itself
            host[:, list(range(k, k + m)) if lost is None else lost] = 0x77
            lay.upload_stripes(host)
    assert (got == ref).all()
    assert _lib.dev().ecamd_bitslice_wait() == 0


def test_background_compiles_queue(sync_compile):
    """Knob 1 (the default): new matrices run on the LDS tables while at most ECAMD_JIT_JOBS (2)
    compiler children build their kernels, the rest queued; every result is exact throughout, and
    once the queue has drained every pass takes the bitsliced kernel -- still exact."""
    k, m, bs, S = 13, 7, 65536, 2
    lay, want = _batch(k, m, bs, S, seed=21)
    pats = [[0, 1, 2, 3, 4, 5, 6], [1, 2, 3, 4, 5, 6, 7], [2, 3, 4, 5, 6, 7, 8], [3, 4, 5, 6, 7, 8, 9],
            [4, 5, 6, 7, 8, 9, 10], [0, 2, 4, 6, 13, 15, 17]]
    sync_compile.ecamd_tune(b"bitslice", 1)
    for rnd in range(2):
        for p in pats:
            host = want.copy()
            host[:, p] = 0xC3
            lay.upload_stripes(host)
            D.rs_decode(k, m, p, lay)
            assert (lay.download_stripes() == want).all(), (rnd, p)
        if rnd == 0:
            assert _lib.dev().ecamd_bitslice_wait() == 0


def test_entries_bounded_and_evicted_kernels_reload(sync_compile):
    """More distinct 8-output matrices than the "bitslice_entries" bound: the least recently used
    are evicted (modules unloaded after their launches drained) and a pattern seen again is
    rebuilt from the disk cache; every result exact."""
    k, m, bs, S = 20, 8, 32768, 2
    lay, want = _batch(k, m, bs, S, seed=31)
    pats = [[j, j + 1, j + 2, j + 3, j + 4, 20, 21, 22] for j in range(5)]
    d = sync_compile
    d.ecamd_tune(b"bitslice_entries", 2)
    try:
        for p in pats + pats[:2]:
            host = want.copy()
            host[:, p] = 0x5C
            lay.upload_stripes(host)
            D.rs_decode(k, m, p, lay)
            assert (lay.download_stripes() == want).all(), p
            assert d.ecamd_bitslice_entries() <= 2
    finally:
        d.ecamd_tune(b"bitslice_entries", 0)


@pytest.mark.parametrize("k,m,lost", [(20, 8, None), (20, 8, [0, 2, 4, 6, 20, 22, 24, 26]), (3, 5, None)])
def test_ring4_many_tiles(sync_compile, k, m, lost):
    """The 4-deep LDS ring (prefetch three inputs ahead, across tile boundaries)."""
    sync_compile.ecamd_tune(b"bitslice_depth", 4)
    _many_tiles(sync_compile, k, m, lost)


@pytest.mark.parametrize("k,m,bs,rows", [(10, 4, 65536 + 100, 4), (6, 3, 49152, 3)])
def test_few_output_builds_exact(sync_compile, k, m, bs, rows):
    """Maps of up to 4 outputs (knob bitslice_min_rows lowered) get the 4-waves-per-SIMD build."""
    d = sync_compile
    d.ecamd_tune(b"bitslice_min_rows", rows)
    try:
        lay, want = _batch(k, m, bs, 3, seed=41)
        D.rs_encode(k, m, lay)
        assert (lay.download_stripes() == want).all()
        lost = list(range(m))
        host = want.copy()
        host[:, lost] = 0x99
        lay.upload_stripes(host)
        D.rs_decode(k, m, lost, lay)
        assert (lay.download_stripes() == want).all()
    finally:
        d.ecamd_tune(b"bitslice_min_rows", 0)


@pytest.mark.parametrize("threads", [128, 512])
@pytest.mark.parametrize("k,m,lost", [(20, 8, None), (20, 8, [0, 2, 4, 6, 20, 22, 24, 26]), (10, 6, [0, 1, 2, 3, 4, 5])])
def test_tile_threads_exact(sync_compile, threads, k, m, lost):
    """The multi-wave form with 128 / 512 lanes per workgroup (8 / 32 KiB tiles, knob bs_tile_threads)
    against the oracle, fragments with a ragged tail (the LDS tables take the rest)."""
    d = sync_compile
    d.ecamd_tune(b"bs_tile_threads", threads)
    try:
        bs = 32768 * 3 + 4096 + 10
        lay, want = _batch(k, m, bs, 3, seed=51)
        if lost is None:
            D.rs_encode(k, m, lay)
        else:
            host = want.copy()
            host[:, lost] = 0x6B
            lay.upload_stripes(host)
            D.rs_decode(k, m, lost, lay)
        assert (lay.download_stripes() == want).all()
    finally:
        d.ecamd_tune(b"bs_tile_threads", 256)
