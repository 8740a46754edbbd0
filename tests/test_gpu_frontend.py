"""GPU tests of liberasurecode.so.1 (B2) through the public C API, restating the reference's
integration suite (test/liberasurecode_test.c TEST_SUITE, :2429-2448) for the backends this build
drives, and checking every fragment byte-for-byte (80-byte header + payload) against a Python
restatement of the framing plus the CPU oracle's parity."""
import ctypes as C
import itertools
import os
import random
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import ec_api as E
import oracle_lib as orc

pytestmark = pytest.mark.gpu

RS_ARGS = [(10, 4), (4, 4), (10, 10), (4, 8), (4, 2), (20, 8)]  # liberasurecode_test.c:252-289 + C2/C5
XOR_ARGS = [(3, 3, 3), (6, 6, 3), (10, 5, 3), (10, 6, 4), (20, 6, 4)]


def payload_bytes(n, seed):
    return random.Random(seed).randbytes(n)


def rs_expected(k, m, data: bytes, ct, legacy=False):
    """Expected k+m fragments for liberasurecode_rs_vand: pad to k*2, split, oracle parity."""
    a = k * 2
    aligned = (len(data) + a - 1) // a * a
    bs = aligned // k
    buf = np.zeros(aligned, dtype=np.uint8)
    buf[:len(data)] = np.frombuffer(data, dtype=np.uint8)
    dfr = buf.reshape(k, bs)
    par = orc.encode(k, m, dfr) if bs else np.zeros((m, 0), np.uint8)
    out = []
    for i in range(k + m):
        p = (dfr[i] if i < k else par[i - k]).tobytes()
        out.append(E.expected_header(i, bs, len(data), E.EC_BACKEND_LIBERASURECODE_RS_VAND, ct, p,
                                     legacy=legacy) + p)
    return out


def xor_expected(k, m, hd, data: bytes, ct):
    import xor_util as X
    a = k * 4
    aligned = (len(data) + a - 1) // a * a
    bs = aligned // k
    buf = np.zeros(aligned, dtype=np.uint8)
    buf[:len(data)] = np.frombuffer(data, dtype=np.uint8)
    dfr = [buf[i * bs:(i + 1) * bs].copy() for i in range(k)]
    pb, _ = X.tables(k, m, hd)
    out = []
    for i in range(k + m):
        if i < k:
            p = dfr[i]
        else:
            p = np.zeros(bs, dtype=np.uint8)
            for j in range(k):
                if pb[i - k] >> j & 1:
                    p ^= dfr[j]
        out.append(E.expected_header(i, bs, len(data), E.EC_BACKEND_FLAT_XOR_HD, ct, p.tobytes())
                   + p.tobytes())
    return out


@pytest.fixture(params=[("rs",) + a for a in RS_ARGS] + [("xor",) + a for a in XOR_ARGS],
                ids=lambda p: "_".join(map(str, p)))
def code(request):
    return request.param


def make(code, ct=E.CHKSUM_NONE):
    if code[0] == "rs":
        _, k, m = code
        desc = E.create(E.EC_BACKEND_LIBERASURECODE_RS_VAND, k, m, hd=m, ct=ct)
        hd = m + 1
    else:
        _, k, m, hd = code
        desc = E.create(E.EC_BACKEND_FLAT_XOR_HD, k, m, hd=hd, ct=ct)
    assert desc > 0, desc
    return desc, k, m, hd


def expected(code, k, m, hd, data, ct, legacy=False):
    if code[0] == "rs":
        return rs_expected(k, m, data, ct, legacy)
    return xor_expected(k, m, hd, data, ct)


@pytest.mark.parametrize("size", [1, 17, 1000, 65536 + 3, 1 << 20])
@pytest.mark.parametrize("ct", [E.CHKSUM_NONE, E.CHKSUM_CRC32])
def test_encode_fragments_byte_exact(code, size, ct):
    desc, k, m, hd = make(code, ct)
    data = payload_bytes(size, size)
    rc, dp, pp, flen = E.encode(desc, data)
    assert rc == 0
    frags = E.fragments(dp, k, flen) + E.fragments(pp, m, flen)
    want = expected(code, k, m, hd, data, ct)
    assert flen == len(want[0])
    for i in range(k + m):
        assert frags[i] == want[i], f"fragment {i}"
    assert E.lib().liberasurecode_encode_cleanup(desc, dp, pp) == 0
    assert E.lib().liberasurecode_instance_destroy(desc) == 0


def _patterns(k, m, hd):
    n = k + m
    maxm = min(hd - 1, m)
    pats = [[i] for i in range(n)]
    pats += [list(p) for p in itertools.combinations(range(n), 2) if maxm >= 2][:60]
    if maxm >= 3:
        pats += [list(range(0, 3)), [0, k, k + 1], [k - 1, k, n - 1]]
    if maxm >= 4:
        pats += [list(range(4)), list(range(k, k + 4))]
    if maxm >= 8:
        pats += [list(range(8)), [0, 2, 4, 6, n - 4, n - 3, n - 2, n - 1]]
    return pats


def test_decode_missing_patterns(code):
    desc, k, m, hd = make(code)
    data = payload_bytes(1 << 20, 99)
    rc, dp, pp, flen = E.encode(desc, data)
    assert rc == 0
    frags = E.fragments(dp, k, flen) + E.fragments(pp, m, flen)
    E.lib().liberasurecode_encode_cleanup(desc, dp, pp)
    for miss in _patterns(k, m, hd):
        avail = [f for i, f in enumerate(frags) if i not in miss]
        rc, out = E.decode(desc, avail, flen, force=1)
        assert rc == 0, miss
        assert out == data, miss
    E.lib().liberasurecode_instance_destroy(desc)


def test_reconstruct_byte_equal(code):
    """reconstruct_test_impl (liberasurecode_test.c:1276-1338): each fragment rebuilt with one more
    fragment missing equals the original fragment INCLUDING its header."""
    desc, k, m, hd = make(code, E.CHKSUM_CRC32)
    data = payload_bytes(300000, 5)
    rc, dp, pp, flen = E.encode(desc, data)
    frags = E.fragments(dp, k, flen) + E.fragments(pp, m, flen)
    E.lib().liberasurecode_encode_cleanup(desc, dp, pp)
    n = k + m
    for extra in ([], [0], [n - 1]):
        for i in range(n):
            gone = set(extra) | {i}
            avail = [f for j, f in enumerate(frags) if j not in gone]
            rc, out = E.reconstruct(desc, avail, flen, i)
            assert rc == 0, (i, extra)
            assert out == frags[i], (i, extra)
    E.lib().liberasurecode_instance_destroy(desc)


def test_fragments_needed_rs():
    desc = E.create(E.EC_BACKEND_LIBERASURECODE_RS_VAND, 10, 4, hd=4)
    rc, needed = E.fragments_needed(desc, [0], [], 14)
    assert rc == 0 and needed == list(range(1, 11))
    rc, needed = E.fragments_needed(desc, [0, 1], [2, 11], 14)
    assert rc == 0 and needed == [3, 4, 5, 6, 7, 8, 9, 10, 12, 13]
    rc, needed = E.fragments_needed(desc, [0, 1, 2], [3, 4], 14)
    assert rc == -1
    E.lib().liberasurecode_instance_destroy(desc)


def test_fragments_needed_xor_first_parity():
    # test_fragments_needed_impl: reconstruct data connected to the first parity (10,5,3)
    desc = E.create(E.EC_BACKEND_FLAT_XOR_HD, 10, 5, hd=3)
    rc, needed = E.fragments_needed(desc, [0], [3], 15)
    assert rc == 0 and needed == [1, 5, 7, 10]  # p0 = {0,1,5,7} (parity bm 163)
    E.lib().liberasurecode_instance_destroy(desc)


def test_metadata_checksums_and_legacy_crc(monkeypatch):
    desc = E.create(E.EC_BACKEND_LIBERASURECODE_RS_VAND, 10, 4, hd=4, ct=E.CHKSUM_CRC32)
    data = payload_bytes(123457, 1)
    rc, dp, pp, flen = E.encode(desc, data)
    frags = E.fragments(dp, 10, flen) + E.fragments(pp, 4, flen)
    E.lib().liberasurecode_encode_cleanup(desc, dp, pp)
    md = E.FragmentMetadata()
    for i, f in enumerate(frags):
        assert E.lib().liberasurecode_get_fragment_metadata(f, C.byref(md)) == 0
        assert md.idx == i and md.chksum_mismatch == 0 and md.chksum_type == E.CHKSUM_CRC32
        assert E.lib().is_invalid_fragment(desc, f) == 0
    bad = bytearray(frags[3])
    bad[100] ^= 0x40  # corrupt the payload: checksum mismatch flagged, header still valid
    assert E.lib().liberasurecode_get_fragment_metadata(bytes(bad), C.byref(md)) == 0
    assert md.chksum_mismatch == 1
    assert E.lib().is_invalid_fragment(desc, bytes(bad)) == 1
    # LIBERASURECODE_WRITE_LEGACY_CRC: headers and payload CRC in the legacy form
    monkeypatch.setenv("LIBERASURECODE_WRITE_LEGACY_CRC", "1")
    rc, dp, pp, flen = E.encode(desc, data)
    leg = E.fragments(dp, 10, flen) + E.fragments(pp, 4, flen)
    E.lib().liberasurecode_encode_cleanup(desc, dp, pp)
    want = rs_expected(10, 4, data, E.CHKSUM_CRC32, legacy=True)
    assert leg == want
    for f in leg:
        assert E.lib().liberasurecode_get_fragment_metadata(f, C.byref(md)) == 0
        assert md.chksum_mismatch == 0
    monkeypatch.delenv("LIBERASURECODE_WRITE_LEGACY_CRC")
    rc, out = E.decode(desc, leg[2:], flen, force=1)
    assert rc == 0 and out == data
    E.lib().liberasurecode_instance_destroy(desc)


def test_verify_stripe_metadata():
    desc = E.create(E.EC_BACKEND_LIBERASURECODE_RS_VAND, 4, 2, hd=2, ct=E.CHKSUM_CRC32)
    rc, dp, pp, flen = E.encode(desc, payload_bytes(4096, 3))
    frags = [C.create_string_buffer(f, flen) for f in E.fragments(dp, 4, flen) + E.fragments(pp, 2, flen)]
    E.lib().liberasurecode_encode_cleanup(desc, dp, pp)
    arr = (C.c_void_p * 6)(*[C.addressof(f) for f in frags])
    assert E.lib().liberasurecode_verify_stripe_metadata(desc, arr, 6) == 0
    assert E.lib().liberasurecode_verify_stripe_metadata(desc, None, 6) == -E.EINVALIDPARAMS
    assert E.lib().liberasurecode_verify_stripe_metadata(desc, arr, 0) == -E.EINVALIDPARAMS
    frags[1][54] = 3  # backend id
    assert E.lib().liberasurecode_verify_stripe_metadata(desc, arr, 6) == -E.EBADHEADER
    frags[1][54] = 6
    frags[2][0] = 7  # idx >= k+m
    assert E.lib().liberasurecode_verify_stripe_metadata(desc, arr, 6) == -E.EBADHEADER
    frags[2][0] = 2
    frags[3][55] = 9  # backend version
    assert E.lib().liberasurecode_verify_stripe_metadata(desc, arr, 6) == -E.EBADHEADER
    frags[3][55] = 0
    frags[4][53] = 1  # chksum_mismatch stored
    assert E.lib().liberasurecode_verify_stripe_metadata(desc, arr, 6) == -E.EBADCHKSUM
    E.lib().liberasurecode_instance_destroy(desc)


def test_invalid_arguments_and_bad_input():
    desc = E.create(E.EC_BACKEND_LIBERASURECODE_RS_VAND, 4, 2, hd=2)
    lib = E.lib()
    d = C.POINTER(C.c_void_p)()
    p = C.POINTER(C.c_void_p)()
    fl = C.c_uint64()
    assert lib.liberasurecode_encode(desc, None, 10, C.byref(d), C.byref(p), C.byref(fl)) == -E.EINVALIDPARAMS
    assert lib.liberasurecode_encode(desc, b"abc", 3, None, C.byref(p), C.byref(fl)) == -E.EINVALIDPARAMS
    assert lib.liberasurecode_encode(9999, b"abc", 3, C.byref(d), C.byref(p), C.byref(fl)) == -E.EBACKENDNOTAVAIL
    rc, dp, pp, flen = E.encode(desc, payload_bytes(1000, 4))
    frags = E.fragments(dp, 4, flen) + E.fragments(pp, 2, flen)
    lib.liberasurecode_encode_cleanup(desc, dp, pp)
    assert E.decode(desc, frags[:3], flen)[0] == -E.EINSUFFFRAGS
    assert E.decode(desc, frags, 79)[0] == -E.EBADHEADER
    bad = bytearray(frags[0])
    bad[60] ^= 1  # magic
    assert E.decode(desc, [bytes(bad)] + frags[1:], flen)[0] == -E.EBADHEADER
    assert E.reconstruct(desc, frags[1:], flen, 0)[0] == 0
    rc, out = E.reconstruct(desc, frags, flen, 2)  # destination supplied: copied through
    assert rc == 0 and out == frags[2]
    assert lib.liberasurecode_reconstruct_fragment(desc, None, 3, flen, 0, C.create_string_buffer(flen)) == -E.EINVALIDPARAMS
    assert lib.liberasurecode_get_aligned_data_size(desc, 1001) == 1008
    assert lib.liberasurecode_get_minimum_encode_size(desc) == 8
    assert lib.liberasurecode_get_fragment_size(desc, 1001) == 252
    lib.liberasurecode_instance_destroy(desc)


def test_unaligned_fragments_realigned():
    desc = E.create(E.EC_BACKEND_LIBERASURECODE_RS_VAND, 10, 4, hd=4)
    data = payload_bytes(50000, 8)
    rc, dp, pp, flen = E.encode(desc, data)
    frags = E.fragments(dp, 10, flen) + E.fragments(pp, 4, flen)
    E.lib().liberasurecode_encode_cleanup(desc, dp, pp)
    raw = [C.create_string_buffer(flen + 16) for _ in frags]
    ptrs = []
    for b, f in zip(raw, frags):
        C.memmove(C.addressof(b) + 3, f, flen)  # 3 bytes off 16-byte alignment
        ptrs.append(C.addressof(b) + 3)
    arr = (C.c_void_p * 10)(*ptrs[4:])
    out = C.c_void_p()
    olen = C.c_uint64()
    assert E.lib().liberasurecode_decode(desc, arr, 10, flen, 0, C.byref(out), C.byref(olen)) == 0
    assert C.string_at(out.value, olen.value) == data
    E.lib().liberasurecode_decode_cleanup(desc, out)
    E.lib().liberasurecode_instance_destroy(desc)


def test_concurrent_calls_share_one_instance():
    """liberasurecode_threaded_test.c: many threads encode / decode / reconstruct on one
    descriptor under the shared read lock; results must stay exact."""
    desc = E.create(E.EC_BACKEND_LIBERASURECODE_RS_VAND, 10, 4, hd=4, ct=E.CHKSUM_CRC32)

    def job(t):
        data = payload_bytes(200000 + t * 1000, t)
        rc, dp, pp, flen = E.encode(desc, data)
        assert rc == 0
        frags = E.fragments(dp, 10, flen) + E.fragments(pp, 4, flen)
        E.lib().liberasurecode_encode_cleanup(desc, dp, pp)
        assert frags == rs_expected(10, 4, data, E.CHKSUM_CRC32)
        rc, out = E.decode(desc, frags[t % 4:t % 4 + 10], flen)
        assert rc == 0 and out == data
        rc, fr = E.reconstruct(desc, frags[1:], flen, 0)
        assert rc == 0 and fr == frags[0]
        return True

    with ThreadPoolExecutor(8) as ex:
        assert all(ex.map(job, range(32)))
    E.lib().liberasurecode_instance_destroy(desc)


@pytest.mark.parametrize("hd", [3, 4])
def test_xor_too_many_failures(hd):
    # test_flat_xor_decode_too_many_failures / _reconstruct_too_many_failures (:1804-1915)
    desc = E.create(E.EC_BACKEND_FLAT_XOR_HD, 5, 5, hd=hd)
    data = payload_bytes(1 << 20, 9)
    rc, dp, pp, flen = E.encode(desc, data)
    frags = E.fragments(dp, 5, flen) + E.fragments(pp, 5, flen)
    E.lib().liberasurecode_encode_cleanup(desc, dp, pp)
    arr = (C.c_char_p * 6)(*frags[4:])
    out = C.c_void_p()
    olen = C.c_uint64()
    assert E.lib().liberasurecode_decode(desc, arr, 6, flen, 1, C.byref(out), C.byref(olen)) == -1
    assert out.value is None and olen.value == 0
    for j in range(5):  # only parity left: the backend fails
        assert E.reconstruct(desc, frags[5:], flen, j)[0] < 0
    for j in range(9):  # one fragment left: the pre-check refuses
        assert E.reconstruct(desc, frags[9:], flen, j)[0] == -E.EINSUFFFRAGS
    E.lib().liberasurecode_instance_destroy(desc)


@pytest.mark.parametrize("zero_all", ["0", "1"])
def test_frontend_on_dirty_heap(zero_all):
    """The frontend zeroes only what this repo's codec does not overwrite (frontend.cpp: lean
    encode buffers, assemble): with glibc handing out garbage-filled memory every fragment and
    every decoded object must still equal the reference framing's (zero padding, zero tail).
    ECAMD_FRONTEND_ZERO_ALL=1 is the reference's full zeroing, the A/B switch."""
    import json
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, MALLOC_PERTURB_="165", MALLOC_MMAP_THRESHOLD_="33554432",
               ECAMD_FRONTEND_ZERO_ALL=zero_all)
    r = subprocess.run([sys.executable, os.path.join(here, "perturbed_heap_run.py")],
                       capture_output=True, text=True, timeout=300, env=env,
                       cwd=os.path.dirname(here))
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["perturbed"], "glibc did not perturb the heap: the test proves nothing"
    assert res["cases"] >= 150
    assert res["failures"] == []


def test_decode_direct_matches_general_path():
    """Encode with the object -> payload copies on the codec's staging pack (tees) and
    liberasurecode_decode straight into the object (frontend.cpp decode_direct: rebuilt data
    unpacked in place, missing parity not rebuilt, surviving payloads copied once) against the
    general path in the reference's order (fresh fragments for every missing index, parity rebuilt,
    fragments_to_string afterwards; ECAMD_FRONTEND_DECODE_DIRECT=0): identical return codes and
    objects for every erasure pattern sampled, and for irregular survivors (another payload size or
    orig_data_size in a data fragment's header, a duplicate fragment), which the direct path hands
    back to the general one."""
    import json
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    res = {}
    # (decode straight into the object, staging-pack tees for the object <-> payload copies)
    for direct, tee in (("1", "1"), ("1", "0"), ("0", "0")):
        env = dict(os.environ, ECAMD_FRONTEND_DECODE_DIRECT=direct, ECAMD_FRONTEND_TEE=tee)
        r = subprocess.run([sys.executable, os.path.join(here, "percall_decode_run.py")], capture_output=True,
                           text=True, timeout=240, env=env)
        assert r.returncode == 0, r.stderr[-3000:]
        res[direct + tee] = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["11"] == res["10"] == res["00"]
    assert all(ok for _, _, _, ok in res["11"] if ok is not None), [x for x in res["11"] if x[3] is False][:5]
    assert sum(1 for _, rc, _, ok in res["11"] if ok) > 100


@pytest.mark.parametrize("legacy", [False, True])
@pytest.mark.parametrize("km", [(10, 4), (4, 2), (20, 8), (10, 6, 4), (3, 3, 3)])
def test_percall_crc_fused(monkeypatch, km, legacy):
    """The per-call CHKSUM_CRC32 encode with the payload checksums folded into the small-launch codec
    kernel (ecamd_map_apply_strided_crc: one launch, inputs staged through LDS, one workgroup or a
    cross-workgroup Horner) -- every fragment byte-equal to the restated framing over zlib / the legacy
    CRC, at sizes from 1 byte to past the small-launch limit (64 KiB fragments), with the fused-launch
    counter proving the path (from 16 KiB of fragments; the host's zlib below); (20, 8) does not fit the
    LDS and must take the separate pass / host."""
    import torch  # noqa: F401  (one HIP runtime per process: torch's)
    from liberasurecode_amd import _lib
    k, m = km[:2]
    xor = len(km) == 3  # flat_xor_hd (k, m, hd): xor_small_kernel's fused checksums
    if xor and legacy:
        pytest.skip("the XOR framing restatement covers the zlib checksum")
    d = _lib.dev()
    cnt = d.ecamd_small_crc_launches
    cnt.restype = C.c_longlong
    if legacy:
        monkeypatch.setenv("LIBERASURECODE_WRITE_LEGACY_CRC", "1")
    desc = (E.create(E.EC_BACKEND_FLAT_XOR_HD, k, m, hd=km[2], ct=E.CHKSUM_CRC32) if xor
            else E.create(E.EC_BACKEND_LIBERASURECODE_RS_VAND, k, m, hd=m, ct=E.CHKSUM_CRC32))
    fused = 0
    for size in (1, 15, 100, 1000, 4096, 4097, 5121, 16384, 16400, 65536 + 3, 200000, 262144, 640000, 655361,
                 1 << 20):
        data = payload_bytes(size, size + k)
        n0 = cnt()
        rc, dp, pp, flen = E.encode(desc, data)
        assert rc == 0
        fused += cnt() - n0
        frags = E.fragments(dp, k, flen) + E.fragments(pp, m, flen)
        E.lib().liberasurecode_encode_cleanup(desc, dp, pp)
        want = (xor_expected(k, m, km[2], data, E.CHKSUM_CRC32) if xor
                else rs_expected(k, m, data, E.CHKSUM_CRC32, legacy=legacy))
        assert frags == want, (size, legacy)
    E.lib().liberasurecode_instance_destroy(desc)
    if km == (20, 8):
        assert fused == 0
    else:
        assert fused >= 3, fused  # the sizes with >= 16 KiB of fragments, each at most 64 KiB
