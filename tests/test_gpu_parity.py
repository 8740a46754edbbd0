"""GPU parity: the HIP path (libecamd.so, liberasurecode_rs_vand.so.1) against the reference's
golden vectors, the C oracle and the independent numpy GF(2^16).  Needs an MI355X."""
import ctypes as C
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

import gfnp
import oracle_lib as orc
from ecdata import EDGE_PATTERNS, stripe_fragments
from liberasurecode_amd import _lib
from liberasurecode_amd import device as D

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "rs_vand.json")))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module", autouse=True)
def _device():
    assert D.available(), _lib.dev().ecamd_last_error()


def _upload(frags_sfb):
    S, F, bs = frags_sfb.shape
    lay = D.Layout.alloc(F, bs, S)
    lay.upload_stripes(frags_sfb)
    return lay


def test_fill_splitmix_matches_numpy():
    lay = D.Layout.alloc(5, 1000, 3)
    lay.fill_splitmix(stripe0=7)
    D.synchronize()
    got = lay.download_stripes()
    for s in range(3):
        assert (got[s] == stripe_fragments(7 + s, 5, 1000)).all()


def _case_data(case):
    k, bs = case["k"], case["bs"]
    if case.get("pattern"):
        return np.stack([EDGE_PATTERNS[case["pattern"]](bs) for _ in range(k)])
    return stripe_fragments(case["stripe"], k, bs)


@pytest.mark.parametrize("case", GOLD["encode"],
                         ids=lambda c: f"{c['k']}-{c['m']}-{c['bs']}-{c['pattern']}")
def test_encode_golden(case):
    k, m, bs = case["k"], case["m"], case["bs"]
    frags = np.zeros((1, k + m, bs), dtype=np.uint8)
    frags[0, :k] = _case_data(case)
    frags[0, k:] = 0xA5  # parity must be overwritten
    lay = _upload(frags)
    D.rs_encode(k, m, lay)
    out = lay.download_stripes()[0]
    assert [sha(out[k + p]) for p in range(m)] == case["parity_sha256"]


def _decode_frags(case):
    k, m, bs = case["k"], case["m"], case["bs"]
    data = stripe_fragments(case["stripe"], k, bs)
    par = (stripe_fragments(case["stripe"], m, bs, base=0xBAD0) if case["garbage"]
           else orc.encode(k, m, data))
    frags = np.concatenate([data, par])[None].copy()
    for i in case["missing"]:
        frags[0, i] = 0x5A  # missing slots are overwritten, whatever they hold
    return frags


@pytest.mark.parametrize("case", GOLD["decode"],
                         ids=lambda c: f"{c['k']}-{c['m']}-{c['bs']}-{c['missing']}-{c['garbage']}")
def test_decode_golden(case):
    k, m = case["k"], case["m"]
    lay = _upload(_decode_frags(case))
    if case["ret"] != 0:
        with pytest.raises(_lib.ECAmdError):
            D.rs_decode(k, m, case["missing"], lay)
        return
    D.rs_decode(k, m, case["missing"], lay)
    out = lay.download_stripes()[0]
    assert {str(i): sha(out[i]) for i in case["missing"]} == case["out_sha256"]


@pytest.mark.parametrize("case", GOLD["reconstruct"],
                         ids=lambda c: f"{c['k']}-{c['m']}-{c['missing']}-{c['dest']}-{c['garbage']}")
def test_reconstruct_golden(case):
    k, m = case["k"], case["m"]
    frags = _decode_frags(case)
    for i in case["missing"]:
        frags[0, i] = 0  # the reference test zeroes missing buffers
    lay = _upload(frags)
    D.rs_reconstruct(k, m, case["missing"], case["dest"], lay)
    out = lay.download_stripes()[0]
    assert sha(out[case["dest"]]) == case["out_sha256"]


@pytest.mark.parametrize("k,m,bs,S", [(4, 2, 65536, 64), (10, 4, 1 << 20, 8), (10, 4, 4096, 257),
                                      (20, 8, 1 << 18, 6), (12, 6, 3000, 33)])
def test_batched_encode_matches_oracle(k, m, bs, S):
    lay = D.Layout.alloc(k + m, bs, S)
    lay.fill_splitmix(nfrags=k, stripe0=100)
    D.rs_encode(k, m, lay)
    out = lay.download_stripes()
    for s in sorted({0, S // 2, S - 1}):
        data = stripe_fragments(100 + s, k, bs)
        assert (out[s, :k] == data).all()
        assert (out[s, k:] == orc.encode(k, m, data)).all()


@pytest.mark.parametrize("tiles_per_slot", [0, 1])
@pytest.mark.parametrize("k,m,bs,S,missing", [
    (10, 4, 1 << 20, 16, [0, 1, 2, 3]), (10, 4, 1 << 20, 16, [0, 5, 10, 13]),
    (20, 8, 1 << 22, 4, list(range(8))), (20, 8, 1 << 20, 4, [0, 2, 4, 6, 20, 22, 24, 26]),
    (4, 2, 65536, 128, [1, 3]), (10, 4, (1 << 20) + 40, 7, [2, 11])])
def test_roundtrip_encode_erase_decode(k, m, bs, S, missing, tiles_per_slot):
    """tiles_per_slot 1: every pass split into launches of at most one tile per resident
    workgroup (a few launches each here), as long batches are split by default."""
    _lib.check(_lib.dev().ecamd_tune(b"tiles_per_slot", tiles_per_slot), "tune")
    try:
        _roundtrip(k, m, bs, S, missing)
    finally:
        _lib.dev().ecamd_tune(b"tiles_per_slot", 0)


def _roundtrip(k, m, bs, S, missing):
    lay = D.Layout.alloc(k + m, bs, S)
    lay.fill_splitmix(nfrags=k, stripe0=5)
    D.rs_encode(k, m, lay)
    ref = lay.download_stripes()
    host = ref.copy()
    host[:, missing] = 0xEE
    lay.upload_stripes(host)
    D.rs_decode(k, m, missing, lay)
    assert (lay.download_stripes() == ref).all()
    # reconstruct each erased fragment on its own, as liberasurecode_reconstruct_fragment does
    for d in missing[:3]:
        lay.upload_stripes(host)
        D.rs_reconstruct(k, m, missing, d, lay)
        assert (lay.download_stripes()[:, d] == ref[:, d]).all()


def test_long_batch_split_into_launches():
    """A batch of more than 64 tiles per resident workgroup runs as several stream launches
    (ecamd_device.hip launch_stream_pass): k=4 m=2, 64 KiB+16 fragments (17 tiles each, the last
    partial), 5000 stripes = 85000 tiles, so at least two launches on a 256-CU MI355X.  Encode
    checked against the oracle on stripes around every possible split, strided decode and the
    stripe-list decode_multi (4000 stripes in one erasure group: split too) on the whole batch."""
    k, m, bs, S = 4, 2, 65536 + 16, 5000
    lay = D.Layout.alloc(k + m, bs, S)
    lay.fill_splitmix(nfrags=k, stripe0=3)
    D.rs_encode(k, m, lay)
    ref = lay.download_stripes()
    rng = np.random.default_rng(7)
    check = {0, 1, S - 2, S - 1} | set(rng.integers(0, S, 12).tolist())
    for cus in (128, 256, 304):  # the split point for other CU counts, 4 workgroups per CU
        b = 64 * cus * 4 // 17
        check |= {b - 1, b, b + 1}
    for s in sorted(x for x in check if 0 <= x < S):
        data = stripe_fragments(3 + s, k, bs)
        assert (ref[s, :k] == data).all()
        assert (ref[s, k:] == orc.encode(k, m, data)).all(), s
    host = ref.copy()
    host[:, [0, 4]] = 0x5A
    lay.upload_stripes(host)
    D.rs_decode(k, m, [0, 4], lay)
    assert (lay.download_stripes() == ref).all()
    pats = [[0, 5] if s % 5 == 0 else [1] for s in range(S)]
    for s, pat in enumerate(pats):
        host[s] = ref[s]
        host[s, pat] = 0xA5
    lay.upload_stripes(host)
    D.rs_decode_multi(k, m, pats, lay)
    assert (lay.download_stripes() == ref).all()
    lay.buf.free()


@pytest.mark.parametrize("streams", [1, 3])
@pytest.mark.parametrize("tiles_per_slot", [0, 1])
@pytest.mark.parametrize("k,m,bs,S", [(10, 4, 65536 + 6, 64), (4, 2, 4096, 200), (20, 8, 8192, 40)])
def test_decode_multi_heterogeneous(k, m, bs, S, tiles_per_slot, streams):
    """Every stripe lost its own set of fragments (including none, all-parity and
    m-missing cases); one call rebuilds them all, each equal to the oracle's decode of that
    stripe on the same (inconsistent, garbage-filled) buffers.  tiles_per_slot 1: the stripe-list
    launches split into several."""
    _lib.check(_lib.dev().ecamd_tune(b"tiles_per_slot", tiles_per_slot), "tune")
    _lib.check(_lib.dev().ecamd_tune(b"multi_streams", streams), "tune")  # per-pattern launches on 3 streams
    try:
        _decode_multi_case(k, m, bs, S)
    finally:
        _lib.dev().ecamd_tune(b"tiles_per_slot", 0)
        _lib.dev().ecamd_tune(b"multi_streams", 1)


def _decode_multi_case(k, m, bs, S):
    rng = np.random.default_rng(k * 100 + S)
    lay = D.Layout.alloc(k + m, bs, S)
    lay.fill_splitmix(nfrags=k, stripe0=9)
    D.rs_encode(k, m, lay)
    host = lay.download_stripes()
    pats = []
    for s in range(S):
        n = int(rng.integers(0, m + 1))
        pat = sorted(rng.choice(k + m, n, replace=False).tolist())
        if s % 7 == 0:
            pat = list(range(k, k + m))  # parity only
        rng.shuffle(pat)
        pats.append(pat)
        host[s, pat] = rng.integers(0, 256, (len(pat), bs), dtype=np.uint8)
    lay.upload_stripes(host)
    D.rs_decode_multi(k, m, pats, lay)
    got = lay.download_stripes()
    for s in range(S):
        frags = [host[s, f].copy() for f in range(k + m)]
        assert orc.decode(k, m, frags, pats[s]) == 0
        assert all((got[s, f] == frags[f]).all() for f in range(k + m)), (s, pats[s])


@pytest.mark.parametrize("bs", [1, 2, 3, 15, 16, 17, 31, 33, 255, 1000, 4097])
@pytest.mark.parametrize("R,K", [(1, 3), (2, 5), (3, 4), (4, 10), (6, 7), (8, 20), (9, 25), (5, 45)])
def test_map_tails_and_shapes(bs, R, K):
    rng = np.random.default_rng(bs * 1000 + R * 10 + K)
    coeff = rng.integers(0, 65536, size=(R, K))
    coeff[0, 0] = 1
    ins = [rng.integers(0, 256, size=bs, dtype=np.uint8) for _ in range(K)]
    frags = np.zeros((2, K + R, bs), dtype=np.uint8)
    frags[:, :K] = np.stack(ins)
    frags[:, K:] = 0x77
    lay = _upload(frags)
    D.GF16Map(coeff).apply(lay, list(range(K)), list(range(K, K + R)))
    out = lay.download_stripes()
    want = gfnp.apply_map(coeff, ins)
    for r in range(R):
        assert (out[0, K + r] == want[r]).all(), (r, bs)
        assert (out[1, K + r] == want[r]).all()


@pytest.mark.parametrize("bs", [8192, 3 * 4096 + 40])
def test_map_apply_pointer_tables(bs):
    k, m, S = 10, 4, 5
    lay = D.Layout.alloc(k + m, bs, S)
    lay.fill_splitmix(nfrags=k)
    G = np.array(orc.generator(k, m)).reshape(k + m, k)
    mp = D.GF16Map(G[k:])
    ptrs = np.array([lay.buf.ptr + s * lay.stripe_stride + f * lay.frag_stride
                     for s in range(S) for f in range(k + m)], dtype=np.uint64)
    pbuf = D.DeviceBuffer(ptrs.nbytes)
    pbuf.upload(ptrs.view(np.uint8))
    rc = _lib.dev().ecamd_map_apply_ptrs(mp.handle, pbuf.ptr, k + m, _lib.ints(range(k)), pbuf.ptr,
                                         k + m, _lib.ints(range(k, k + m)), bs, S, None)
    assert rc == 0
    out = lay.download_stripes()
    for s in range(S):
        assert (out[s, k:] == orc.encode(k, m, out[s, :k])).all()


@pytest.mark.parametrize("bs", [16, 1000, 4096, 65536 + 3])
def test_xor_apply(bs):
    rng = np.random.default_rng(bs)
    K, R, S = 6, 3, 4
    frags = rng.integers(0, 256, size=(S, K + R, bs), dtype=np.uint8)
    lay = _upload(frags)
    masks = [0b101001, 0b010110, 0b111111]
    D.xor_apply(masks, lay, list(range(K)), list(range(K, K + R)))
    out = lay.download_stripes()
    for r, mk in enumerate(masks):
        want = np.zeros((S, bs), dtype=np.uint8)
        for j in range(K):
            if mk >> j & 1:
                want ^= frags[:, j]
        assert (out[:, K + r] == want).all()


# ---------------------------------------------------------------- drop-in B1 .so ----

def _b1():
    lib = C.CDLL(os.path.join(ROOT, "liberasurecode_amd", "lib", "liberasurecode_rs_vand.so.1"))
    IP = C.POINTER(C.c_int)
    lib.make_systematic_matrix.restype = IP
    lib.make_systematic_matrix.argtypes = [C.c_int, C.c_int]
    lib.liberasurecode_rs_vand_encode.argtypes = [IP, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int]
    lib.liberasurecode_rs_vand_decode.argtypes = [IP, C.c_void_p, C.c_void_p, C.c_int, C.c_int, IP,
                                                  C.c_int, C.c_int]
    lib.liberasurecode_rs_vand_reconstruct.argtypes = [IP, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                                       IP, C.c_int, C.c_int]
    return lib


def test_b1_abi_golden():
    lib = _b1()
    for case in GOLD["encode"][:12]:
        k, m, bs = case["k"], case["m"], case["bs"]
        lib.init_liberasurecode_rs_vand(k, m)
        G = lib.make_systematic_matrix(k, m)
        assert bool(G)
        data = [np.array(x) for x in _case_data(case)]
        par = [np.full(bs, 0xA5, dtype=np.uint8) for _ in range(m)]
        lib.liberasurecode_rs_vand_encode(G, orc.ptr_array(data), orc.ptr_array(par), k, m, bs)
        assert [sha(p) for p in par] == case["parity_sha256"]
    for case in GOLD["decode"]:
        if case["bs"] > 65536:
            continue
        k, m = case["k"], case["m"]
        G = lib.make_systematic_matrix(k, m)
        frags = [np.array(x) for x in _decode_frags(case)[0]]
        rc = lib.liberasurecode_rs_vand_decode(G, orc.ptr_array(frags[:k]), orc.ptr_array(frags[k:]),
                                               k, m, orc.ints(case["missing"] + [-1]), case["bs"], 1)
        assert rc == case["ret"]
        if rc == 0:
            assert {str(i): sha(frags[i]) for i in case["missing"]} == case["out_sha256"]
    for case in GOLD["reconstruct"]:
        if case["bs"] > 65536:
            continue
        k, m = case["k"], case["m"]
        G = lib.make_systematic_matrix(k, m)
        frags = [np.array(x) for x in _decode_frags(case)[0]]
        for i in case["missing"]:
            frags[i][:] = 0
        rc = lib.liberasurecode_rs_vand_reconstruct(G, orc.ptr_array(frags[:k]),
                                                    orc.ptr_array(frags[k:]), k, m,
                                                    orc.ints(case["missing"] + [-1]), case["dest"],
                                                    case["bs"])
        assert rc == case["ret"]
        assert sha(frags[case["dest"]]) == case["out_sha256"]


def test_reference_unit_test_runs_on_our_codec():
    """The reference's own test/builtin/rs_vand/liberasurecode_rs_vand_test.c, compiled from its
    source by oracle/Makefile, run against OUR liberasurecode_rs_vand.so.1 via LD_LIBRARY_PATH."""
    exe = os.path.join(ROOT, "oracle", "_ref", "liberasurecode_rs_vand_test")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref not built (needs the reference sources at build time)")
    env = dict(os.environ, LD_LIBRARY_PATH=os.path.join(ROOT, "liberasurecode_amd", "lib"))
    probe = subprocess.run(["ldd", exe], env=env, capture_output=True, text=True).stdout
    assert os.path.join("liberasurecode_amd", "lib", "liberasurecode_rs_vand.so.1") in probe
    r = subprocess.run([exe], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


def test_scatter_fragments_single_device():
    """ecamd_scatter_fragments with every destination on this device (the one-GPU box): each
    fragment column lands, stripe by stripe, at its own strided destination."""
    k, m, bs, S = 10, 4, 4096 + 80, 6
    lay = D.Layout.alloc(k + m, bs, S)
    lay.fill_splitmix()
    src = lay.download_stripes()
    dsts = [D.DeviceBuffer(S * (bs + 32 * f + 16)) for f in range(k + m)]
    strides = [bs + 32 * f + 16 for f in range(k + m)]
    d = _lib.dev()
    f = d.ecamd_scatter_fragments
    f.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_void_p,
                  C.c_void_p, C.c_void_p, C.c_void_p]
    assert f(lay.buf.ptr, lay.stripe_stride, lay.frag_stride, bs, k + m, S, _lib.ints([0] * (k + m)),
             (C.c_void_p * (k + m))(*[b.ptr for b in dsts]), _lib.i64s(strides), None) == 0
    D.synchronize()
    for i in range(k + m):
        got = dsts[i].download(S * strides[i]).reshape(S, strides[i])[:, :bs]
        assert (got == src[:, i]).all(), i
    assert f(lay.buf.ptr, lay.stripe_stride, lay.frag_stride, bs, 1, S, _lib.ints([7]),
             (C.c_void_p * 1)(dsts[0].ptr), _lib.i64s([strides[0]]), None) != 0


# ------------------------------------------- stream kernels vs the first-version kernels ----

@pytest.fixture
def tune():
    d = _lib.dev()
    yield d.ecamd_tune
    for key, val in ((b"stream", 1), (b"stream_ch", 1), (b"stream_pf", 0), (b"stream_nib", 0),
                     (b"stream_order", 0), (b"stream_hybrid", 1), (b"multi_list", 1), (b"xor_wgs", 0),
                     (b"bitslice", 1), (b"small_chunks", -1), (b"small_lane", 0), (b"small_stage", -1)):
        d.ecamd_tune(key, val)


@pytest.mark.parametrize("small", [(0, 0, 1), (1 << 20, 0, 1), (1 << 20, 0, 0), (1 << 20, 4, 1), (1 << 20, 16, 1),
                                   (1 << 20, 16, 0), (1 << 20, 2, 1), (1 << 20, 2, 0)])
@pytest.mark.parametrize("S", [1, 3])
@pytest.mark.parametrize("bs", [1, 15, 16, 17, 416, 1000, 4097, 16384 + 48])
@pytest.mark.parametrize("R,K", [(1, 1), (2, 5), (4, 10), (3, 4), (8, 20), (5, 45), (9, 25)])
def test_small_kernel_shapes(tune, R, K, bs, S, small):
    """gf16_small_kernel (launches of few chunks: per-call objects) and, with small_chunks 0, the
    stream kernel's tail path on the same shapes, against the numpy GF(2^16) reference: ragged
    fragments, several stripes, 2 / 4 / 8-output passes, K = 45 in column passes (accumulate); the
    small kernel with 2 / 4 bytes per lane by size (default), 4, 16 and 2, its one-stripe launches
    with the inputs staged into LDS first (small_stage 1, default) and read in place (0)."""
    tune(b"small_chunks", small[0])
    tune(b"small_lane", small[1])
    tune(b"small_stage", small[2])
    rng = np.random.default_rng(bs * 7 + R * 100 + K + S)
    coeff = rng.integers(0, 65536, size=(R, K))
    frags = rng.integers(0, 256, size=(S, K + R, bs), dtype=np.uint8)
    lay = _upload(frags)
    D.GF16Map(coeff).apply(lay, list(range(K)), list(range(K, K + R)))
    out = lay.download_stripes()
    for s in range(S):
        want = gfnp.apply_map(coeff, [frags[s, j] for j in range(K)])
        for r in range(R):
            assert (out[s, K + r] == want[r]).all(), (s, r)
        assert (out[s, :K] == frags[s, :K]).all()


def test_small_kernel_nonuniform_offsets(tune):
    """Inputs in a permuted order (no uniform pitch): the small launch declines, the result stays
    exact; the same map with the inputs in order takes it."""
    K, R, bs = 6, 3, 700
    rng = np.random.default_rng(5)
    coeff = rng.integers(0, 65536, size=(R, K))
    frags = rng.integers(0, 256, size=(1, K + R, bs), dtype=np.uint8)
    order = [3, 0, 5, 1, 4, 2]
    for ins in (order, list(range(K))):
        lay = _upload(frags)
        D.GF16Map(coeff).apply(lay, ins, list(range(K, K + R)))
        out = lay.download_stripes()
        want = gfnp.apply_map(coeff, [frags[0, j] for j in ins])
        for r in range(R):
            assert (out[0, K + r] == want[r]).all(), (ins, r)


@pytest.mark.parametrize("S,stage", [(2, 1), (1, 1), (1, 0)])
@pytest.mark.parametrize("small", [0, 1 << 20])
@pytest.mark.parametrize("bs", [1, 3, 4, 17, 416, 4097])
@pytest.mark.parametrize("R,K", [(1, 1), (3, 6), (4, 10), (10, 32)])
def test_xor_small_kernel(tune, R, K, bs, small, S, stage):
    """xor_small_kernel (flat XOR launches of few chunks) and the stream kernel on the same shapes,
    1 and 2 stripes: ragged fragments, more than 8 outputs (row groups), 32 inputs (the masks' width);
    one-stripe launches with the inputs staged into LDS (small_stage 1, default) or read in place."""
    tune(b"small_chunks", small)
    tune(b"small_stage", stage)
    rng = np.random.default_rng(bs * 3 + R * 50 + K)
    frags = rng.integers(0, 256, size=(S, K + R, bs), dtype=np.uint8)
    masks = [int(m) | 1 << (r % K) for r, m in enumerate(rng.integers(0, 1 << min(K, 62), size=R, dtype=np.int64))]
    masks = [m & 0xFFFFFFFF for m in masks]
    lay = _upload(frags)
    D.xor_apply(masks, lay, list(range(K)), list(range(K, K + R)))
    out = lay.download_stripes()
    for r, mk in enumerate(masks):
        want = np.zeros((S, bs), dtype=np.uint8)
        for j in range(K):
            if mk >> j & 1:
                want ^= frags[:, j]
        assert (out[:, K + r] == want).all(), r


@pytest.mark.parametrize("R,K", [(1, 1), (2, 4), (2, 5), (4, 10), (4, 13), (7, 16), (8, 20), (3, 21)])
@pytest.mark.parametrize("variant", [(b"stream", 0), (b"stream", 1), (b"stream_pf", 1),
                                     (b"stream_nib", 1), (b"stream_ch", 2), (b"stream_order", 1),
                                     (b"stream_hybrid", 0), (b"bitslice", 0)])
def test_stream_kernel_variants(tune, R, K, variant):
    """Every gf16 kernel variant (the stream kernel and its tuning knobs, the first-version kernel,
    K = 21 falling back to it) against the numpy GF(2^16) reference on full 4 KiB tiles plus a
    ragged tail, 3 stripes."""
    tune(*variant)
    bs = 3 * 4096 + 48
    rng = np.random.default_rng(R * 100 + K)
    coeff = rng.integers(0, 65536, size=(R, K))
    frags = rng.integers(0, 256, size=(3, K + R, bs), dtype=np.uint8)
    lay = _upload(frags)
    D.GF16Map(coeff).apply(lay, list(range(K)), list(range(K, K + R)))
    out = lay.download_stripes()
    for s in range(3):
        want = gfnp.apply_map(coeff, [frags[s, j] for j in range(K)])
        for r in range(R):
            assert (out[s, K + r] == want[r]).all(), (s, r)


@pytest.mark.parametrize("stream,multi_list", [(0, 0), (1, 0), (1, 1)])
@pytest.mark.parametrize("k,m,bs,S", [(10, 4, 65536 + 6, 24), (20, 8, 8192 + 2, 10), (24, 4, 4096 + 10, 6)])
def test_decode_multi_pointer_kernels(tune, stream, multi_list, k, m, bs, S):
    """Heterogeneous batch decode on the stripe-list stream launches, the pointer-table stream
    kernel and the first-version pointer kernel, checked against the oracle on garbage-filled
    buffers."""
    tune(b"stream", stream)
    tune(b"multi_list", multi_list)
    rng = np.random.default_rng(k * 7 + stream)
    host = rng.integers(0, 256, size=(S, k + m, bs), dtype=np.uint8)
    for s in range(S):
        host[s, k:] = orc.encode(k, m, host[s, :k])
    pats = [sorted(rng.choice(k + m, size=int(rng.integers(1, m + 1)), replace=False).tolist())
            for _ in range(S)]
    dirty = host.copy()
    for s in range(S):
        for f in pats[s]:
            dirty[s, f] = rng.integers(0, 256, size=bs, dtype=np.uint8)
    lay = _upload(dirty)
    D.rs_decode_multi(k, m, pats, lay)
    got = lay.download_stripes()
    assert (got == host).all()


@pytest.mark.parametrize("K", [1, 3, 4, 7, 12, 17, 32])
@pytest.mark.parametrize("stream", [0, 1])
def test_xor_stream_kernel(tune, K, stream):
    tune(b"stream", stream)
    R, S, bs = 5, 3, 2 * 4096 + 1040
    rng = np.random.default_rng(K)
    frags = rng.integers(0, 256, size=(S, K + R, bs), dtype=np.uint8)
    masks = [int(x) for x in rng.integers(0, 1 << K, size=R)]
    lay = _upload(frags)
    D.xor_apply(masks, lay, list(range(K)), list(range(K, K + R)))
    out = lay.download_stripes()
    for r, mk in enumerate(masks):
        want = np.zeros((S, bs), dtype=np.uint8)
        for j in range(K):
            if mk >> j & 1:
                want ^= frags[:, j]
        assert (out[:, K + r] == want).all(), r


def test_fragment_major_layout_beyond_2gib():
    """Fragment-major layout [k+m][S][bs] whose fragment offsets pass 2 GiB: the stream kernel's
    32-bit buffer offsets do not reach, so the launch falls back to the 64-bit-address kernel.
    Encode and a decode of the data stripes, checked against the oracle at both ends."""
    k, m, bs = 4, 2, 4096
    S = (1 << 31) // bs + 8  # frag_stride = S*bs > 2 GiB
    buf = D.DeviceBuffer((k + m) * S * bs)
    lay = D.Layout(buf, k + m, bs, S, frag_stride=S * bs, stripe_stride=bs)
    lay.fill_splitmix(nfrags=k)
    D.rs_encode(k, m, lay)
    D.synchronize()

    def stripe(s):
        return np.stack([buf.download(bs, f * S * bs + s * bs) for f in range(k + m)])

    for s in (0, S - 1):
        got = stripe(s)
        assert (got[:k] == stripe_fragments(s, k, bs)).all()
        assert (got[k:] == orc.encode(k, m, got[:k])).all(), s
    want = stripe(S - 1)
    D.rs_decode(k, m, [0, 3], lay)
    D.synchronize()
    assert (stripe(S - 1) == want).all()
    buf.free()
