"""GPU: the reference's API test suite (test/liberasurecode_test.c), restated in Python against the
drop-in liberasurecode.so.1 for the two backends this build serves.

The reference's own file cannot be compiled here (it includes the autoconf-generated
config_liberasurecode.h), so each test below follows one of its functions line for line -- same
argument tables (liberasurecode_rs_vand_test_args, flat_xor_test_args, :78-85, :252-289), same
skip patterns, same assertions -- and cites it.  A checksummed (CRC32) variant of every argument
set is added, since the reference's tables only use CHKSUM_NONE.
"""
import ctypes as C
import os

import pytest

import ec_api as E
import oracle_lib as O

pytestmark = pytest.mark.gpu

RS = E.EC_BACKEND_LIBERASURECODE_RS_VAND
XOR = E.EC_BACKEND_FLAT_XOR_HD
# (backend, k, m, w, hd), test/liberasurecode_test.c:78-85, 252-289
ARGS = [(RS, 10, 4, 16, 5), (RS, 4, 4, 16, 5), (RS, 10, 10, 16, 11), (RS, 4, 8, 16, 9),
        (XOR, 3, 3, 0, 3)]
CASES = [(a, ct) for a in ARGS for ct in (E.CHKSUM_NONE, E.CHKSUM_CRC32)]
IDS = [f"{'rs' if a[0] == RS else 'xor'}_{a[1]}_{a[2]}_ct{ct}" for a, ct in CASES]
HDR = 80
ORIG = 1024 * 1024


def create(a, ct):
    be, k, m, w, hd = a
    desc = E.create(be, k, m, hd=hd, ct=ct, w=w)
    assert desc > 0, desc
    return desc


def encode(desc, data, k, m):
    rc, d, p, flen = E.encode(desc, data)
    assert rc == 0
    frags = E.fragments(d, k, flen) + E.fragments(p, m, flen)
    assert E.lib().liberasurecode_encode_cleanup(desc, d, p) == 0
    return frags, flen


def avail(frags, skip):
    """create_frags_array (:85-117): every fragment whose skip flag is 0, data then parity."""
    return [f for i, f in enumerate(frags) if not skip[i]]


def meta(frag):
    md = E.FragmentMetadata()
    C.memmove(C.addressof(md), frag, 59)
    return md


def encode_decode_test_impl(a, ct, skip):
    """encode_decode_test_impl (:1180-1274)."""
    be, k, m = a[0], a[1], a[2]
    desc = create(a, ct)
    orig = os.urandom(ORIG)
    frags, flen = encode(desc, orig, k, m)
    remaining, off = ORIG, 0
    for i, frag in enumerate(frags):
        md = meta(frag)
        assert md.idx == i
        assert md.size == flen - HDR - md.frag_backend_metadata_size
        assert md.orig_data_size == ORIG
        assert md.backend_id == be
        assert md.chksum_mismatch == 0
        cmp = min(remaining, md.size)
        assert frag[HDR:HDR + cmp] == orig[off:off + cmp]
        remaining -= cmp
        off += md.size
    rc, out = E.decode(desc, avail(frags, skip), flen, force=1)
    assert rc == 0 and out == orig
    assert E.lib().liberasurecode_instance_destroy(desc) == 0


def reconstruct_test_impl(a, ct, skip):
    """reconstruct_test_impl (:1276-1338): every fragment rebuilt byte-equal, header included."""
    k, m = a[1], a[2]
    desc = create(a, ct)
    frags, flen = encode(desc, os.urandom(ORIG), k, m)
    for i in range(k + m):
        s = list(skip)
        s[i] = 1
        rc, out = E.reconstruct(desc, avail(frags, s), flen, i)
        assert rc == 0
        assert out == frags[i], i
    assert E.lib().liberasurecode_instance_destroy(desc) == 0


@pytest.mark.parametrize("a,ct", CASES, ids=IDS)
def test_simple_encode_decode(a, ct):
    """:1980-1987"""
    encode_decode_test_impl(a, ct, [0] * (a[1] + a[2]))


@pytest.mark.parametrize("a,ct", CASES, ids=IDS)
def test_simple_reconstruct(a, ct):
    """:2004-2024"""
    reconstruct_test_impl(a, ct, [0] * (a[1] + a[2]))


@pytest.mark.parametrize("a,ct", CASES, ids=IDS)
def test_decode_with_missing_data(a, ct):
    """:1556-1569"""
    k, m = a[1], a[2]
    for i in range(k):
        skip = [0] * (k + m)
        skip[i] = 1
        encode_decode_test_impl(a, ct, skip)


@pytest.mark.parametrize("a,ct", CASES, ids=IDS)
def test_decode_with_missing_parity(a, ct):
    """:1571-1584"""
    k, m = a[1], a[2]
    for i in range(k, k + m):
        skip = [0] * (k + m)
        skip[i] = 1
        encode_decode_test_impl(a, ct, skip)


@pytest.mark.parametrize("a,ct", CASES, ids=IDS)
def test_decode_with_missing_multi_data(a, ct):
    """:1586-1605: windows of min(k, hd-1) data fragments (wrapping inside the data)."""
    k, m, hd = a[1], a[2], a[4]
    mx = k if k <= hd - 1 else hd - 1
    for i in range(k - mx + 1):
        skip = [0] * (k + m)
        for j in range(i, i + mx):
            skip[j % k] = 1
        encode_decode_test_impl(a, ct, skip)


@pytest.mark.parametrize("a,ct", CASES, ids=IDS)
def test_decode_with_missing_multi_parity(a, ct):
    """:1607-1621"""
    k, m, hd = a[1], a[2], a[4]
    mx = hd - 1
    for i in range(k, k + m - mx + 1):
        skip = [0] * (k + m)
        for j in range(i, i + mx):
            skip[j] = 1
        encode_decode_test_impl(a, ct, skip)


@pytest.mark.parametrize("a,ct", CASES, ids=IDS)
def test_decode_with_missing_multi_data_parity(a, ct):
    """:1623-1641"""
    k, m, hd = a[1], a[2], a[4]
    mx = hd - 1
    for i in range(k + m - mx + 1):
        skip = [0] * (k + m)
        for j in range(i, i + mx):
            skip[j] = 1
        encode_decode_test_impl(a, ct, skip)


@pytest.mark.parametrize("a", ARGS, ids=[i.rsplit("_ct", 1)[0] for i in IDS[::2]])
def test_fragments_needed_impl(a):
    """:1340-1466: rebuilding a data fragment of the first parity's equation needs that parity
    and the other data fragments of the equation."""
    k, m = a[1], a[2]
    desc = create(a, E.CHKSUM_NONE)
    rc, needed = E.fragments_needed(desc, [k], [], k + m)
    assert rc > -1
    recon = needed[0]
    exclude = next(i for i in range(k + m) if i not in needed[1:])
    rc, new = E.fragments_needed(desc, [recon], [exclude], k + m)
    assert rc > -1
    for f in new:
        assert f == k or f in needed[1:], (needed, new)
    E.lib().liberasurecode_instance_destroy(desc)


def get_fragment_metadata_impl(a, ct, legacy):
    """test_get_fragment_metadata (:1468-1536) with validate_fragment_checksum (:552-585)."""
    be, k, m = a[0], a[1], a[2]
    desc = create(a, ct)
    frags, flen = encode(desc, os.urandom(ORIG), k, m)
    lib = E.lib()
    lib.get_libec_version.argtypes = [C.c_char_p, C.POINTER(C.c_uint32)]
    lib.get_backend_id.argtypes = [C.c_char_p, C.POINTER(C.c_int)]
    lib.get_backend_version.argtypes = [C.c_char_p, C.POINTER(C.c_uint32)]
    for frag in frags:
        md = E.FragmentMetadata()
        C.memset(C.addressof(md), 0xFF, 59)
        assert lib.liberasurecode_get_fragment_metadata(frag, C.byref(md)) == 0
        assert md.orig_data_size == ORIG
        assert md.size != 0
        assert md.chksum_type == ct
        payload = frag[HDR:HDR + md.size]
        if ct == E.CHKSUM_CRC32:
            want = O.crc32(payload, legacy=legacy)
            assert md.chksum[0] == want
        else:
            assert md.chksum_mismatch == 0
        ver, bid, bver = C.c_uint32(), C.c_int(), C.c_uint32()
        assert lib.get_libec_version(frag, C.byref(ver)) == 0 and ver.value == E.LIBEC_VERSION
        assert lib.get_backend_id(frag, C.byref(bid)) == 0 and bid.value == be
        assert lib.get_backend_version(frag, C.byref(bver)) == 0 and bver.value == E.BACKEND_VERSION
    lib.liberasurecode_instance_destroy(desc)


@pytest.mark.parametrize("a,ct", CASES, ids=IDS)
def test_get_fragment_metadata(a, ct):
    get_fragment_metadata_impl(a, ct, legacy=False)


@pytest.mark.parametrize("a", [ARGS[1], ARGS[4]], ids=["rs_4_4", "xor_3_3"])
def test_write_legacy_fragment_metadata(a, monkeypatch):
    """:1538-1554: "1" and "true" write the legacy CRC; "0", "00" and unset do not."""
    for value, legacy in (("1", True), ("true", True), ("0", False), ("00", False), (None, False)):
        if value is None:
            monkeypatch.delenv("LIBERASURECODE_WRITE_LEGACY_CRC", raising=False)
        else:
            monkeypatch.setenv("LIBERASURECODE_WRITE_LEGACY_CRC", value)
        # "00" is not "0": the reference writes the legacy CRC for it (only "" and "0" are off)
        if value == "00":
            legacy = True
        get_fragment_metadata_impl(a, E.CHKSUM_CRC32, legacy)


MISMATCH = ["libec_version", "magic", "backend_id", "backend_version", "idx_invalid",
            "idx_out_of_range", "idx_at_boundary"]


@pytest.mark.parametrize("a", ARGS, ids=[i.rsplit("_ct", 1)[0] for i in IDS[::2]])
@pytest.mark.parametrize("scenario", MISMATCH)
def test_verify_stripe_metadata_mismatch(a, scenario):
    """verify_fragment_metadata_mismatch_impl (:2066-2160) and the tests built on it
    (:2162-2184, 2231-2237): every corrupted fragment is invalid; healed, it is valid again."""
    k, m = a[1], a[2]
    desc = create(a, E.CHKSUM_NONE)
    frags, flen = encode(desc, os.urandom(1024), k, m)
    lib = E.lib()
    bufs = [C.create_string_buffer(f, flen) for f in frags]
    arr = (C.c_void_p * len(bufs))(*[C.addressof(b) for b in bufs])
    assert lib.liberasurecode_verify_stripe_metadata(desc, arr, len(bufs)) == 0
    for b in bufs:
        raw = bytearray(b.raw)
        orig = bytes(raw[:HDR])
        if scenario == "libec_version":
            v = int.from_bytes(raw[63:67], "little") + 1
            raw[63:67] = v.to_bytes(4, "little")
        elif scenario == "magic":
            raw[59:63] = b"\0\0\0\0"
        elif scenario == "backend_id":
            raw[54] = (raw[54] + 1) & 0xFF
        elif scenario == "backend_version":
            v = int.from_bytes(raw[55:59], "little") + 1
            raw[55:59] = v.to_bytes(4, "little")
        elif scenario == "idx_invalid":
            raw[0:4] = (0xFFFFFFFF).to_bytes(4, "little")
        elif scenario == "idx_out_of_range":
            raw[0:4] = (k + m + 1).to_bytes(4, "little")
        else:
            raw[0:4] = (k + m).to_bytes(4, "little")
        C.memmove(b, bytes(raw[:HDR]), HDR)
        assert lib.is_invalid_fragment(desc, b.raw) == 1, scenario
        C.memmove(b, orig, HDR)
        assert lib.is_invalid_fragment(desc, b.raw) == 0
    lib.liberasurecode_instance_destroy(desc)


def test_verify_fragment_metadata_idx_bounds():
    """:2194-2229"""
    desc = E.create(RS, 3, 2, ct=E.CHKSUM_NONE)
    assert desc > 0
    lib = E.lib()
    be = lib.liberasurecode_backend_instance_get_by_desc(desc)
    assert be
    md = E.FragmentMetadata()
    md.backend_id = RS
    md.backend_version = E.BACKEND_VERSION
    md.idx = 4
    assert lib.liberasurecode_verify_fragment_metadata(be, C.byref(md)) == 0
    md.idx = 5
    assert lib.liberasurecode_verify_fragment_metadata(be, C.byref(md)) != 0
    md.idx = 6
    assert lib.liberasurecode_verify_fragment_metadata(be, C.byref(md)) != 0
    lib.liberasurecode_instance_destroy(desc)


def test_reconstruct_corrupt_payload_size():
    """:854-917 on rs_vand (the reference runs it on the null backend, absent here): a first
    surviving fragment claiming a negative payload size, with a pre-1.2.0 version so its header
    checksum is not consulted, makes reconstruct fail with -EBADHEADER."""
    a = (RS, 10, 4, 16, 5)
    desc = create(a, E.CHKSUM_NONE)
    frags, flen = encode(desc, os.urandom(ORIG), 10, 4)
    bad = bytearray(frags[1])
    bad[4:8] = (0xFFFFFFFF).to_bytes(4, "little")   # meta.size
    bad[63:67] = (1).to_bytes(4, "little")          # libec_version below 1.2.0
    avail_frags = [bytes(bad)] + frags[2:]
    rc, _ = E.reconstruct(desc, avail_frags, flen, 0)
    assert rc == -E.EBADHEADER
    E.lib().liberasurecode_instance_destroy(desc)


def test_flat_xor_can_reconstruct_with_many_failures():
    """:1916-1978: with more than k fragments gone, (3,3,hd3) still rebuilds what its equations
    allow."""
    a = (XOR, 3, 3, 0, 3)
    desc = create(a, E.CHKSUM_NONE)
    frags, flen = encode(desc, os.urandom(ORIG), 3, 3)
    skip = [0, 0, 1, 1, 1, 1]
    rc, out = E.reconstruct(desc, avail(frags, skip), flen, 5)
    assert rc == 0 and out == frags[5]
    rc, _ = E.reconstruct(desc, avail(frags, skip), flen, 4)
    assert rc < 1
    skip = [1, 0, 0, 1, 1, 1]
    rc, out = E.reconstruct(desc, avail(frags, skip), flen, 4)
    assert rc == 0 and out == frags[4]
    E.lib().liberasurecode_instance_destroy(desc)
