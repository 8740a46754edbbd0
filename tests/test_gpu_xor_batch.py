"""GPU: flat_xor_hd on strided device batches (ecamd_xor_encode / _decode / _reconstruct /
_decode_multi) against the buffer-level oracle (oracle/xor_oracle.py, the reference's
xor_code.c / xor_hd_code.c restated) on inconsistent random buffers, ragged block sizes.

The batch API reads missing slots as zero -- the frontend hands the codec zero-filled buffers
(src/erasurecode_preprocessing.c:141-147, 180-186) -- so the oracle runs on copies whose missing
slots are zeroed."""
import os
import sys

import numpy as np
import pytest

import xor_util as X

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import xor_oracle as XO  # noqa: E402

CODES = [(3, 3, 3, 4096 + 10), (10, 6, 4, 65536 + 6), (15, 6, 3, 12346), (20, 6, 4, 3000),
         (10, 5, 3, 1 << 16)]


@pytest.fixture(scope="module")
def D():
    import torch  # noqa: F401  (one HIP runtime per process: torch's)
    from liberasurecode_amd import device
    return device


def _batch(D, k, m, bs, S, seed):
    rng = np.random.default_rng(seed)
    host = rng.integers(0, 256, size=(S, k + m, bs), dtype=np.uint8)
    lay = D.Layout.alloc(k + m, bs, S)
    lay.upload_stripes(host)
    return host, lay


def _zeroed(stripe, missing):
    bufs = [x.copy() for x in stripe]
    for i in missing:
        bufs[i][:] = 0
    return bufs


def _recoverable(k, m, hd, seed, n):
    oc = XO.XorCode(k, m, hd)
    pats = X.xor_patterns(k + m, seed)
    rng = np.random.default_rng(seed)
    out = []
    for i in rng.permutation(len(pats)):
        p = pats[int(i)]
        if len(p) < hd and oc.decode([np.zeros(4, np.uint8) for _ in range(k + m)], p, 1) == 0:
            out.append(p)
        if len(out) == n:
            break
    return out


@pytest.mark.parametrize("k,m,hd,bs", CODES)
def test_xor_batch_encode(D, k, m, hd, bs):
    S = 5
    host, lay = _batch(D, k, m, bs, S, k * 31 + bs)
    D.xor_encode(k, m, hd, lay)
    got = lay.download_stripes()
    oc = XO.XorCode(k, m, hd)
    for s in range(S):
        want = [x.copy() for x in host[s]]
        for j in range(k, k + m):
            want[j][:] = 0  # xor_code_encode accumulates into zeroed parity
        oc.encode(want)
        assert all((got[s, i] == want[i]).all() for i in range(k + m)), s


@pytest.mark.parametrize("k,m,hd,bs", CODES)
def test_xor_batch_decode_and_reconstruct(D, k, m, hd, bs):
    S = 3
    oc = XO.XorCode(k, m, hd)
    for p in _recoverable(k, m, hd, 5 + k, 4):
        host, lay = _batch(D, k, m, bs, S, len(p) * 101 + bs)
        D.xor_decode(k, m, hd, p, lay, decode_parity=True)
        got = lay.download_stripes()
        for s in range(S):
            want = _zeroed(host[s], p)
            assert oc.decode(want, p, 1) == 0
            assert all((got[s, i] == want[i]).all() for i in range(k + m)), (p, s)
        dest = p[0]
        host, lay = _batch(D, k, m, bs, S, len(p) * 103 + bs)
        D.xor_reconstruct(k, m, hd, p, dest, lay)
        got = lay.download_stripes()
        for s in range(S):
            want = _zeroed(host[s], p)
            assert oc.reconstruct_one(want, p, dest) == 0
            assert (got[s, dest] == want[dest]).all(), (p, dest, s)


@pytest.mark.parametrize("k,m,hd,bs", CODES)
def test_xor_batch_decode_multi_heterogeneous(D, k, m, hd, bs):
    """Every stripe its own erasure list (some repeated, one stripe with none): one stripe-list
    launch per distinct list, each stripe equal to the oracle's decode of it."""
    S = 12
    oc = XO.XorCode(k, m, hd)
    pats = _recoverable(k, m, hd, 77 + k, 5)
    per = [pats[s % len(pats)] for s in range(S)]
    per[3] = []
    host, lay = _batch(D, k, m, bs, S, 4242 + k)
    D.xor_decode_multi(k, m, hd, per, lay, decode_parity=True)
    got = lay.download_stripes()
    for s in range(S):
        want = _zeroed(host[s], per[s])
        if per[s]:
            assert oc.decode(want, per[s], 1) == 0
        assert all((got[s, i] == want[i]).all() for i in range(k + m)), (s, per[s])


def test_xor_batch_rejects_bad_codes_and_patterns(D):
    from liberasurecode_amd._lib import ECAmdError
    host, lay = _batch(D, 3, 3, 64, 1, 1)
    with pytest.raises(ECAmdError):
        D.xor_encode(3, 4, 3, lay)  # not a flat_xor_hd code
    with pytest.raises(ECAmdError):
        D.xor_decode(3, 3, 3, [0, 1, 2, 3], lay)  # beyond what hd = 3 recovers


def test_xor_batch_split_into_launches(D):
    """Flat-XOR passes split into several launches (knob xor_tiles_per_slot 1: at most one 4 KiB
    tile per resident workgroup per launch -- 40 stripes of 17 tiles take 2 launches on a 256-CU
    MI355X): encode and the stripe-list decode_multi, every stripe against the oracle."""
    from liberasurecode_amd import _lib
    k, m, hd, bs, S = 10, 6, 4, 65536 + 6, 40
    oc = XO.XorCode(k, m, hd)
    _lib.check(_lib.dev().ecamd_tune(b"xor_tiles_per_slot", 1), "tune")
    try:
        host, lay = _batch(D, k, m, bs, S, 99)
        D.xor_encode(k, m, hd, lay)
        got = lay.download_stripes()
        for s in range(S):
            want = [x.copy() for x in host[s]]
            for j in range(k, k + m):
                want[j][:] = 0
            oc.encode(want)
            assert all((got[s, i] == want[i]).all() for i in range(k + m)), s
        pats = _recoverable(k, m, hd, 123, 2)
        per = [pats[0] if s % 8 else pats[1] for s in range(S)]  # 35 stripes in one list: split
        host, lay = _batch(D, k, m, bs, S, 100)
        D.xor_decode_multi(k, m, hd, per, lay, decode_parity=True)
        got = lay.download_stripes()
        for s in range(S):
            want = _zeroed(host[s], per[s])
            assert oc.decode(want, per[s], 1) == 0
            assert all((got[s, i] == want[i]).all() for i in range(k + m)), (s, per[s])
    finally:
        _lib.dev().ecamd_tune(b"xor_tiles_per_slot", -1)
