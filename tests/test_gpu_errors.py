"""Codec failures through liberasurecode.so.1 (B2).

1. Execution failures of this repo's GPU codec (staging allocation, copy, launch) must fail the
   API call with a negative code and hand out no fragments.  The reference frontend checks
   `ret < 0` after every backend call (src/erasurecode.c:454-461, 677-683, 898-904); its rs_vand
   shim discards the codec's return code (src/backends/rs_vand/liberasurecode_rs_vand.c:86-90)
   because a CPU codec cannot fail mid-call.  Faults are injected with ecamd_fault_inject.
2. Codec REFUSALS keep the reference behaviour: k fragments with duplicate indices leave more than
   m fragments missing, liberasurecode_rs_vand_decode / _reconstruct return -1 before writing
   (src/builtin/rs_vand/liberasurecode_rs_vand.c:444-447, 502-505), the shim discards that, and the
   frontend assembles the zero-filled missing slots it allocated
   (src/erasurecode_preprocessing.c:141-147).  The expected bytes below restate exactly that.
"""
import ctypes as C
import errno

import numpy as np
import pytest

import ec_api as E
from liberasurecode_amd import _lib

pytestmark = pytest.mark.gpu


def inject(count):
    d = _lib.dev()
    d.ecamd_fault_inject.argtypes = [C.c_char_p, C.c_int]
    assert d.ecamd_fault_inject(b"staging", count) == 0


@pytest.fixture(params=[("rs", 10, 4, 5), ("rs", 20, 8, 9), ("xor", 3, 3, 3), ("xor", 10, 6, 4)],
                ids=lambda p: "_".join(map(str, p)))
def inst(request):
    kind, k, m, hd = request.param
    backend = E.EC_BACKEND_LIBERASURECODE_RS_VAND if kind == "rs" else E.EC_BACKEND_FLAT_XOR_HD
    desc = E.create(backend, k, m, hd=hd, ct=E.CHKSUM_CRC32)
    assert desc > 0
    yield kind, desc, k, m
    inject(0)
    assert E.lib().liberasurecode_instance_destroy(desc) == 0


def test_encode_execution_failure_is_reported(inst):
    kind, desc, k, m = inst
    data = np.random.default_rng(1).integers(0, 256, 1 << 20, dtype=np.uint8).tobytes()
    inject(1)
    rc, dp, pp, flen = E.encode(desc, data)
    assert rc == -errno.EIO
    assert not dp and not pp, "no fragments may be handed out after a failed encode"
    # the fault was one-shot: the next call succeeds
    rc, dp, pp, flen = E.encode(desc, data)
    assert rc == 0
    E.lib().liberasurecode_encode_cleanup(desc, dp, pp)


def test_decode_and_reconstruct_execution_failure_are_reported(inst):
    kind, desc, k, m = inst
    data = np.random.default_rng(2).integers(0, 256, 3 << 20, dtype=np.uint8).tobytes()
    rc, dp, pp, flen = E.encode(desc, data)
    assert rc == 0
    frags = E.fragments(dp, k, flen) + E.fragments(pp, m, flen)
    E.lib().liberasurecode_encode_cleanup(desc, dp, pp)
    avail = frags[1:]  # data fragment 0 lost: decode needs the codec
    inject(1)
    rc, out = E.decode(desc, avail, flen)
    assert rc == -errno.EIO and out is None
    inject(1)
    rc, frag = E.reconstruct(desc, avail, flen, 0)
    assert rc == -errno.EIO
    # no fault armed: both succeed and are byte-exact
    rc, out = E.decode(desc, avail, flen)
    assert rc == 0 and out == data
    rc, frag = E.reconstruct(desc, avail, flen, 0)
    assert rc == 0 and frag == frags[0]


def _rs_codec():
    k, m = 10, 4
    desc = E.create(E.EC_BACKEND_LIBERASURECODE_RS_VAND, k, m, ct=E.CHKSUM_NONE)
    assert desc > 0
    return desc, k, m


def test_duplicate_fragments_decode_zero_fill_like_reference():
    desc, k, m = _rs_codec()
    try:
        data = np.random.default_rng(3).integers(0, 256, 10 << 16, dtype=np.uint8).tobytes()
        rc, dp, pp, flen = E.encode(desc, data)
        assert rc == 0
        frags = E.fragments(dp, k, flen) + E.fragments(pp, m, flen)
        E.lib().liberasurecode_encode_cleanup(desc, dp, pp)
        bs = flen - 80
        # k fragments, 5 distinct (0, 1, 2, 3, 10): 9 missing > m, the codec refuses
        avail = [frags[0]] * 4 + [frags[1], frags[2], frags[3], frags[10], frags[0], frags[1]]
        assert len(avail) == k
        for _ in range(3):  # fresh (unzeroed) heap buffers must still come back as zeros
            rc, out = E.decode(desc, avail, flen)
            assert rc == 0
            want = b"".join(frags[i][80:] if i < 4 else b"\0" * bs for i in range(k))[:len(data)]
            assert out == want
    finally:
        E.lib().liberasurecode_instance_destroy(desc)


def test_duplicate_fragments_reconstruct_zero_fill_like_reference():
    desc, k, m = _rs_codec()
    try:
        data = np.random.default_rng(4).integers(0, 256, 10 << 16, dtype=np.uint8).tobytes()
        rc, dp, pp, flen = E.encode(desc, data)
        assert rc == 0
        frags = E.fragments(dp, k, flen) + E.fragments(pp, m, flen)
        E.lib().liberasurecode_encode_cleanup(desc, dp, pp)
        bs = flen - 80
        avail = [frags[0]] * 5 + [frags[1], frags[2], frags[11], frags[12], frags[13]]
        for dest in (4, 10):
            rc, frag = E.reconstruct(desc, avail, flen, dest)
            assert rc == 0
            orig = len(data)
            want = E.expected_header(dest, bs, orig, E.EC_BACKEND_LIBERASURECODE_RS_VAND,
                                     E.CHKSUM_NONE, b"\0" * bs) + b"\0" * bs
            assert frag == want
    finally:
        E.lib().liberasurecode_instance_destroy(desc)
