"""The reference's invalid-argument API tests (test/liberasurecode_test.c:598-1072), restated for the
backends this build serves.

The reference runs them on EC_BACKEND_NULL (libnullcode.so.1, out of scope here: the null backend
reports "not available", exactly as the reference does without that library); every function below
takes (backend, k, m, hd) instead and keeps the reference's calls, return codes and order.  They
run in-process on the GPU (tests/test_gpu_reference_api.py, this repo's codecs) and, through
tests/ref_api_invalid_run.py, on the CPU in front of the REFERENCE codec libraries (oracle/_ref) --
the argument checks are the frontend's, so both must hold.

Where the reference passes a descriptor it assumes is unused (`desc = 1`), a descriptor that was
created and destroyed is used instead: in one test process earlier tests may hold descriptor 1."""
import ctypes as C
import os

import ec_api as E

EC_BACKENDS_MAX = 11  # include/erasurecode/erasurecode.h:43-56
HDR = 80
ORIG = 1024 * 1024


def _create(a, ct=E.CHKSUM_NONE):
    be, k, m, hd = a
    desc = E.create(be, k, m, hd=hd, ct=ct)
    assert desc > 0, desc
    return desc


def _dead_desc(a):
    """A descriptor that no instance holds (created, then destroyed)."""
    d = _create(a)
    assert E.lib().liberasurecode_instance_destroy(d) == 0
    return d


def _encode(desc):
    orig = os.urandom(ORIG)  # create_buffer (:440-455)
    rc, d, p, flen = E.encode(desc, orig)
    assert rc == 0, rc
    return orig, d, p, flen


def create_and_destroy_multiple_backends(a):
    """test_create_and_destroy_multiple_backends (:598-615), plus the reference's TODO: desc2 still
    works after desc1 is destroyed."""
    be, k, m, _ = a
    lib = E.lib()
    desc1 = _create(a)
    desc2 = _create(a)
    assert desc1 != desc2
    assert lib.liberasurecode_instance_destroy(desc1) == 0
    orig, d, p, flen = _encode(desc2)
    frags = E.fragments(d, k, flen) + E.fragments(p, m, flen)
    assert lib.liberasurecode_encode_cleanup(desc2, d, p) == 0
    assert E.decode(desc2, frags[1:], flen) == (0, orig)
    assert lib.liberasurecode_instance_destroy(desc2) == 0


def backend_available_invalid_args(a):
    """test_backend_available_invalid_args (:621-626); test_backend_available (:617-619) on this
    backend (the reference asks it of EC_BACKEND_NULL)."""
    lib = E.lib()
    assert lib.liberasurecode_backend_available(EC_BACKENDS_MAX) == 0
    assert lib.liberasurecode_backend_available(a[0]) == 1


def create_backend_invalid_args(a):
    """test_create_backend_invalid_args (:628-655)."""
    be = a[0]
    lib = E.lib()
    args = E.ECArgs(k=a[1], m=a[2], hd=a[3], ct=E.CHKSUM_NONE)
    assert lib.liberasurecode_instance_create(-1, C.byref(args)) == -E.EBACKENDNOTSUPP
    assert lib.liberasurecode_instance_create(EC_BACKENDS_MAX, C.byref(args)) == -E.EBACKENDNOTSUPP
    assert lib.liberasurecode_instance_create(be, None) == -E.EINVALIDPARAMS
    for k, m in ((1000, 1000), (-1, 4), (10, -1)):
        bad = E.ECArgs(k=k, m=m)
        assert lib.liberasurecode_instance_create(be, C.byref(bad)) == -E.EINVALIDPARAMS, (k, m)


def destroy_backend_invalid_args(a):
    """test_destroy_backend_invalid_args (:657-671)."""
    lib = E.lib()
    assert lib.liberasurecode_instance_destroy(-1) < 0
    assert lib.liberasurecode_instance_destroy(_dead_desc(a)) < 0
    desc = _create(a)
    assert lib.liberasurecode_instance_destroy(desc) == 0
    assert lib.liberasurecode_instance_destroy(desc) < 0


class BackendCommon(C.Structure):
    """struct ec_backend_common (include/erasurecode/erasurecode_backend.h:119-131), the head of
    struct ec_backend."""
    _fields_ = [("id", C.c_int), ("name", C.c_char * 64), ("soname", C.c_char_p),
                ("soversion", C.c_char * 64), ("ops", C.c_void_p), ("ec_backend_version", C.c_uint32)]


ENCODE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int)


def encode_invalid_args(a):
    """test_encode_invalid_args (:673-722), including the encode_failure_stub swapped into the
    instance's ops table (:546-550, :712-718): a failing backend encode fails the call."""
    lib = E.lib()
    orig = os.urandom(ORIG)
    d = C.POINTER(C.c_void_p)()
    p = C.POINTER(C.c_void_p)()
    flen = C.c_uint64()
    assert lib.liberasurecode_encode(-1, orig, ORIG, C.byref(d), C.byref(p), C.byref(flen)) < 0
    desc = _create(a)
    assert lib.liberasurecode_encode(desc, None, ORIG, C.byref(d), C.byref(p), C.byref(flen)) < 0
    assert lib.liberasurecode_encode(desc, orig, ORIG, None, C.byref(p), C.byref(flen)) < 0
    assert lib.liberasurecode_encode(desc, orig, ORIG, C.byref(d), None, C.byref(flen)) < 0
    assert lib.liberasurecode_encode(desc, orig, ORIG, C.byref(d), C.byref(p), None) < 0
    # instance->common.ops->encode = encode_failure_stub (struct ec_backend_op_stubs: init, exit,
    # is_systematic, encode -- include/erasurecode/erasurecode_backend.h:76-80)
    inst = lib.liberasurecode_backend_instance_get_by_desc(desc)
    assert inst
    ops = C.c_void_p.from_address(inst + BackendCommon.ops.offset).value
    slot = C.c_void_p.from_address(ops + 3 * 8)
    saved = slot.value
    stub = ENCODE_FN(lambda *_: -1)
    slot.value = C.cast(stub, C.c_void_p).value
    try:
        assert lib.liberasurecode_encode(desc, orig, ORIG, C.byref(d), C.byref(p), C.byref(flen)) < 0
    finally:
        slot.value = saved
    rc, d2, p2, fl2 = E.encode(desc, orig)  # restored: works again
    assert rc == 0 and lib.liberasurecode_encode_cleanup(desc, d2, p2) == 0
    lib.liberasurecode_instance_destroy(desc)


def encode_cleanup_invalid_args(a):
    """test_encode_cleanup_invalid_args (:724-754)."""
    lib = E.lib()
    desc = _create(a)
    _, d, p, _ = _encode(desc)
    assert lib.liberasurecode_encode_cleanup(-1, d, p) < 0
    assert lib.liberasurecode_encode_cleanup(desc, None, None) == 0
    assert lib.liberasurecode_encode_cleanup(desc, d, p) == 0
    lib.liberasurecode_instance_destroy(desc)


def _decode_raw(desc, frags, n, flen, force, out=True, out_len=True):
    lib = E.lib()
    arr = None if frags is None else (C.c_char_p * len(frags))(*frags)
    o, ol = C.c_void_p(), C.c_uint64()
    return lib.liberasurecode_decode(desc, arr, n, flen, force, C.byref(o) if out else None,
                                     C.byref(ol) if out_len else None)


def decode_invalid_args(a):
    """test_decode_invalid_args (:756-852): header-less fake fragments (create_fake_frags_no_meta,
    :471-497) are -EBADHEADER with force_metadata_checks 1 and 0 and with fragment_len 1; fewer than
    k fragments are -EINSUFFFRAGS before any is read; then the NULL and bad-descriptor cases."""
    _, k, m, _ = a
    lib = E.lib()
    desc = _create(a)
    fake_len = 1024
    fakes = [os.urandom(fake_len) for _ in range(k + m)]
    assert _decode_raw(desc, fakes, k + m, fake_len, 1) == -E.EBADHEADER
    assert _decode_raw(desc, fakes, k + m, fake_len, 0) == -E.EBADHEADER
    assert _decode_raw(desc, fakes, k + m, 1, 1) == -E.EBADHEADER
    short = [os.urandom(1) for _ in range(k - 1)]
    if k - 1 > 0:
        assert _decode_raw(desc, short, k - 1, fake_len, 1) == -E.EINSUFFFRAGS
    _, d, p, flen = _encode(desc)
    frags = E.fragments(d, k, flen) + E.fragments(p, m, flen)
    assert _decode_raw(-1, frags, k + m, flen, 1) < 0
    assert _decode_raw(desc, None, k + m, flen, 1) < 0
    assert _decode_raw(desc, frags, k + m, flen, 1, out=False) < 0
    assert _decode_raw(desc, frags, k + m, flen, 1, out_len=False) < 0
    lib.liberasurecode_encode_cleanup(desc, d, p)
    lib.liberasurecode_instance_destroy(desc)


def decode_cleanup_invalid_args(a):
    """test_decode_cleanup_invalid_args (:919-939)."""
    lib = E.lib()
    buf = C.create_string_buffer(1024)
    assert lib.liberasurecode_decode_cleanup(_dead_desc(a), buf) < 0
    desc = _create(a)
    assert lib.liberasurecode_decode_cleanup(desc, None) == 0
    lib.liberasurecode_instance_destroy(desc)


def reconstruct_fragment_invalid_args(a):
    """test_reconstruct_fragment_invalid_args (:941-991), -EINSUFFFRAGS from one valid fragment."""
    _, k, m, _ = a
    lib = E.lib()
    frag_len = 10
    small = [C.create_string_buffer(frag_len) for _ in range(2)]
    avail = (C.c_void_p * 2)(*[C.addressof(b) for b in small])
    out = C.create_string_buffer(frag_len)
    f = lib.liberasurecode_reconstruct_fragment
    assert f(_dead_desc(a), avail, 1, frag_len, 1, out) < 0
    desc = _create(a)
    assert f(desc, None, 1, frag_len, 1, out) < 0
    assert f(desc, avail, 1, frag_len, 1, None) < 0
    _, d, p, flen = _encode(desc)
    out = C.create_string_buffer(flen)
    assert f(desc, d, 1, flen, 1, out) == -E.EINSUFFFRAGS
    lib.liberasurecode_encode_cleanup(desc, d, p)
    lib.liberasurecode_instance_destroy(desc)


def fragments_needed_invalid_args(a):
    """test_fragments_needed_invalid_args (:993-1020)."""
    lib = E.lib()
    recon, excl, needed = C.c_int(-1), C.c_int(-1), (C.c_int * 64)()
    f = lib.liberasurecode_fragments_needed
    assert f(_dead_desc(a), C.byref(recon), C.byref(excl), needed) < 0
    desc = _create(a)
    assert f(desc, None, C.byref(excl), needed) < 0
    assert f(desc, C.byref(recon), None, needed) < 0
    assert f(desc, C.byref(recon), C.byref(excl), None) < 0
    lib.liberasurecode_instance_destroy(desc)


def get_fragment_metadata_invalid_args(a=None):
    """test_get_fragment_metadata_invalid_args (:1022-1044); needs no instance."""
    lib = E.lib()
    frag = bytearray(1024)
    frag[59:63] = E.MAGIC.to_bytes(4, "little")
    md = E.FragmentMetadata()
    assert lib.liberasurecode_get_fragment_metadata(None, C.byref(md)) < 0
    assert lib.liberasurecode_get_fragment_metadata(bytes(frag), None) < 0
    assert lib.liberasurecode_get_fragment_metadata(bytes(1024), C.byref(md)) == -E.EBADHEADER


def verify_stripe_metadata_invalid_args(a):
    """test_verify_stripe_metadata_invalid_args (:1046-1072)."""
    lib = E.lib()
    n = 6
    frags = (C.c_void_p * n)()
    f = lib.liberasurecode_verify_stripe_metadata
    assert f(-1, frags, n) == -E.EINVALIDPARAMS
    desc = _create(a)
    assert f(desc, None, n) == -E.EINVALIDPARAMS
    assert f(desc, frags, -1) == -E.EINVALIDPARAMS
    assert f(desc, frags, 0) == -E.EINVALIDPARAMS
    lib.liberasurecode_instance_destroy(desc)


def reconstruct_destination_out_of_range(a):
    """DEVIATION: a destination_idx outside [0, k+m) is -EINVALIDPARAMS here.
    The reference does not check it and indexes parity[destination_idx - k] past the array
    (src/erasurecode.c:857-862, undefined behaviour)."""
    _, k, m, _ = a
    lib = E.lib()
    desc = _create(a)
    orig, d, p, flen = _encode(desc)
    frags = E.fragments(d, k, flen) + E.fragments(p, m, flen)
    lib.liberasurecode_encode_cleanup(desc, d, p)
    for dest in (-1, k + m, k + m + 7):
        rc, _ = E.reconstruct(desc, frags[1:], flen, dest)
        assert rc == -E.EINVALIDPARAMS, (dest, rc)
    rc, got = E.reconstruct(desc, frags[1:], flen, 0)  # in range: still works
    assert rc == 0 and got == frags[0]
    lib.liberasurecode_instance_destroy(desc)


SUITE = [create_and_destroy_multiple_backends, backend_available_invalid_args,
         create_backend_invalid_args, destroy_backend_invalid_args, encode_invalid_args,
         encode_cleanup_invalid_args, decode_invalid_args, decode_cleanup_invalid_args,
         reconstruct_fragment_invalid_args, fragments_needed_invalid_args,
         get_fragment_metadata_invalid_args, verify_stripe_metadata_invalid_args,
         reconstruct_destination_out_of_range]

# (backend, k, m, hd): rs_vand (10,4) as liberasurecode_rs_vand_test_args (:252-256) and flat_xor_hd
# (3,3,3) as flat_xor_test_args (:78-83)
BACKENDS = {"rs": (E.EC_BACKEND_LIBERASURECODE_RS_VAND, 10, 4, 5),
            "xor": (E.EC_BACKEND_FLAT_XOR_HD, 3, 3, 3)}
