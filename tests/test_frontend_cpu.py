"""CPU tests of liberasurecode.so.1 (B2): header / checksum logic pinned by the reference's own
known-answer headers (test/liberasurecode_test.c:2239-2315), argument checking, and loud failure
of instance creation when no GPU is present."""
import ctypes as C
import os
import zlib

import pytest

import ec_api as E

HAS_GPU = os.path.exists("/dev/kfd")

# test/liberasurecode_test.c:2242-2246 (little-endian header written with the legacy crc32)
LE_HEADER = bytes.fromhex(
    "0300000000000400000000000000100000000000010000000000000000000000"
    "000000000000000000000000000000000000000000000701" "0e0200cc5e0c0b00"
    "04010022ee45b9000000000000000000")
# test/liberasurecode_test.c:2281-2285 (big-endian)
BE_HEADER = bytes.fromhex(
    "0000000300040000000000000000000000100000010000000000000000000000"
    "000000000000000000000000000000000000000000000700" "020e010b0c5ecc00"
    "010400fa85407000000000000000000000")[:80]


def test_header_sizes():
    assert len(LE_HEADER) == 80 and len(BE_HEADER) == 80


@pytest.mark.parametrize("hdr,zlib_bytes", [
    (LE_HEADER, {70: 0x18, 69: 0x73, 68: 0xF8, 67: 0xEC}),
    (BE_HEADER, {67: 0xE3, 68: 0x73, 69: 0x88, 70: 0xA0})])
def test_metadata_crcs_known_answers(hdr, zlib_bytes):
    lib = E.lib()
    md = E.FragmentMetadata()
    buf = C.create_string_buffer(hdr, 80)
    assert lib.liberasurecode_get_fragment_metadata(buf, C.byref(md)) == 0
    assert buf.raw[:80] == hdr
    assert md.backend_version == (2 << 16) | (14 << 8) | 1
    assert lib.is_invalid_fragment_header(buf) == 0
    # switch the stored metadata checksum to zlib's value
    h = bytearray(hdr)
    for off, v in zlib_bytes.items():
        h[off] = v
    buf = C.create_string_buffer(bytes(h), 80)
    assert lib.liberasurecode_get_fragment_metadata(buf, C.byref(md)) == 0
    assert md.backend_version == (2 << 16) | (14 << 8) | 1
    assert lib.is_invalid_fragment_header(buf) == 0
    # a wrong checksum
    h[70] = 0xFF
    buf = C.create_string_buffer(bytes(h), 80)
    assert lib.liberasurecode_get_fragment_metadata(buf, C.byref(md)) == -E.EBADHEADER
    assert lib.is_invalid_fragment_header(buf) == 1


def test_crc32_alt_matches_restatement():
    lib = E.lib()
    for data in (b"", b"a", b"123456789", bytes(range(256)) * 3, b"\xff" * 1000):
        got = lib.liberasurecode_crc32_alt(0, data, len(data)) & 0xFFFFFFFF
        assert got == E.crc32_legacy(data)
    # the legacy value differs from zlib exactly when a high bit propagates
    assert E.crc32_legacy(b"123456789") != zlib.crc32(b"123456789")


def test_version_and_availability():
    lib = E.lib()
    assert lib.liberasurecode_get_version() == E.LIBEC_VERSION
    for bid in (1, 2, 4, 5, 7, 8, 9, 10, 11, 99):
        assert lib.liberasurecode_backend_available(bid) == 0
    assert lib.liberasurecode_backend_available(E.EC_BACKEND_LIBERASURECODE_RS_VAND) == 1
    assert lib.liberasurecode_backend_available(E.EC_BACKEND_FLAT_XOR_HD) == 1


def test_create_argument_errors():
    lib = E.lib()
    assert lib.liberasurecode_instance_create(E.EC_BACKEND_LIBERASURECODE_RS_VAND, None) == -E.EINVALIDPARAMS
    assert E.create(99, 4, 2) == -E.EBACKENDNOTSUPP
    assert E.create(E.EC_BACKEND_LIBERASURECODE_RS_VAND, -1, 2) == -E.EINVALIDPARAMS
    assert E.create(E.EC_BACKEND_LIBERASURECODE_RS_VAND, 200, 57) == -E.EINVALIDPARAMS
    assert E.create(1, 4, 2) == -E.EBACKENDNOTAVAIL  # jerasure: not built here
    assert lib.liberasurecode_instance_destroy(12345) == -E.EBACKENDNOTAVAIL


@pytest.mark.skipif(HAS_GPU, reason="checks the no-GPU behaviour")
def test_create_fails_loudly_without_gpu():
    assert E.create(E.EC_BACKEND_LIBERASURECODE_RS_VAND, 10, 4) == -E.EBACKENDINITERR
    assert E.create(E.EC_BACKEND_FLAT_XOR_HD, 3, 3, hd=3) == -E.EBACKENDINITERR


def test_fragment_partition_and_helpers():
    lib = E.lib()
    frags = []
    for idx in (0, 2, 5):
        h = E.expected_header(idx, 16, 40, 6, E.CHKSUM_NONE, b"")
        frags.append(C.create_string_buffer(h + b"\0" * 16, 96))
    k, m = 4, 2
    data = (C.c_void_p * k)()
    parity = (C.c_void_p * m)()
    missing = (C.c_int * (k + m))(*([-1] * (k + m)))
    arr = (C.c_void_p * 3)(*[C.addressof(f) for f in frags])
    assert lib.get_fragment_partition(k, m, arr, 3, data, parity, missing) == 0
    assert list(missing) == [1, 3, 4, -1, -1, -1]
    ver = C.c_uint32()
    assert lib.get_libec_version(frags[0], C.byref(ver)) == 0 and ver.value == E.LIBEC_VERSION
    bid = C.c_int()
    assert lib.get_backend_id(frags[0], C.byref(bid)) == 0 and bid.value == 6
