"""ctypes binding of liberasurecode.so.1 (include/erasurecode.h) + a Python restatement of the
80-byte fragment header (include/erasurecode/erasurecode.h:254-324 of the reference) used as the
framing oracle in tests."""
import ctypes as C
import os
import struct
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "liberasurecode_amd", "lib", "liberasurecode.so.1")

EC_BACKEND_NULL, EC_BACKEND_FLAT_XOR_HD, EC_BACKEND_LIBERASURECODE_RS_VAND = 0, 3, 6
CHKSUM_NONE, CHKSUM_CRC32, CHKSUM_MD5 = 1, 2, 3
EBACKENDNOTSUPP, EECMETHODNOTIMPL, EBACKENDINITERR, EBACKENDINUSE, EBACKENDNOTAVAIL = 200, 201, 202, 203, 204
EBADCHKSUM, EINVALIDPARAMS, EBADHEADER, EINSUFFFRAGS = 205, 206, 207, 208
MAGIC = 0xB0C5ECC
LIBEC_VERSION = (1 << 16) | (8 << 8)
BACKEND_VERSION = 1 << 16


class Reserved(C.Structure):
    _fields_ = [("x", C.c_uint64), ("y", C.c_uint64), ("z", C.c_uint64), ("a", C.c_uint64)]


class Priv(C.Union):
    _fields_ = [("reserved", Reserved)]


class ECArgs(C.Structure):
    _fields_ = [("k", C.c_int), ("m", C.c_int), ("w", C.c_int), ("hd", C.c_int),
                ("priv_args1", Priv), ("priv_args2", C.c_void_p), ("ct", C.c_int)]


class FragmentMetadata(C.Structure):
    _pack_ = 1
    _fields_ = [("idx", C.c_uint32), ("size", C.c_uint32), ("frag_backend_metadata_size", C.c_uint32),
                ("orig_data_size", C.c_uint64), ("chksum_type", C.c_uint8),
                ("chksum", C.c_uint32 * 8), ("chksum_mismatch", C.c_uint8),
                ("backend_id", C.c_uint8), ("backend_version", C.c_uint32)]


assert C.sizeof(FragmentMetadata) == 59

_lib = None


def lib():
    global _lib
    if _lib is None:
        l = C.CDLL(LIB)
        CPP = C.POINTER(C.c_char_p)
        l.liberasurecode_instance_create.argtypes = [C.c_int, C.POINTER(ECArgs)]
        l.liberasurecode_encode.argtypes = [C.c_int, C.c_char_p, C.c_uint64,
                                            C.POINTER(C.POINTER(C.c_void_p)),
                                            C.POINTER(C.POINTER(C.c_void_p)), C.POINTER(C.c_uint64)]
        l.liberasurecode_encode_cleanup.argtypes = [C.c_int, C.c_void_p, C.c_void_p]
        l.liberasurecode_decode.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_uint64, C.c_int,
                                            C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]
        l.liberasurecode_decode_cleanup.argtypes = [C.c_int, C.c_void_p]
        l.liberasurecode_reconstruct_fragment.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_uint64,
                                                          C.c_int, C.c_char_p]
        l.liberasurecode_fragments_needed.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        l.liberasurecode_get_fragment_metadata.argtypes = [C.c_char_p, C.POINTER(FragmentMetadata)]
        l.is_invalid_fragment_header.argtypes = [C.c_char_p]
        l.is_invalid_fragment.argtypes = [C.c_int, C.c_char_p]
        l.liberasurecode_verify_stripe_metadata.argtypes = [C.c_int, C.c_void_p, C.c_int]
        l.liberasurecode_get_aligned_data_size.argtypes = [C.c_int, C.c_uint64]
        l.liberasurecode_get_fragment_size.argtypes = [C.c_int, C.c_int]
        l.liberasurecode_get_version.restype = C.c_uint32
        l.liberasurecode_crc32_alt.argtypes = [C.c_int, C.c_char_p, C.c_size_t]
        l.liberasurecode_backend_instance_get_by_desc.restype = C.c_void_p
        l.liberasurecode_verify_fragment_metadata.argtypes = [C.c_void_p, C.POINTER(FragmentMetadata)]
        _lib = l
    return _lib


def create(backend, k, m, hd=0, ct=CHKSUM_NONE, w=0):
    a = ECArgs(k=k, m=m, w=w, hd=hd, ct=ct)
    return lib().liberasurecode_instance_create(backend, C.byref(a))


def encode(desc, data: bytes):
    d = C.POINTER(C.c_void_p)()
    p = C.POINTER(C.c_void_p)()
    flen = C.c_uint64()
    rc = lib().liberasurecode_encode(desc, data, len(data), C.byref(d), C.byref(p), C.byref(flen))
    return rc, d, p, flen.value


def fragments(ptrs, n, flen):
    return [C.string_at(ptrs[i], flen) for i in range(n)]


def decode(desc, frags, flen, force=0):
    arr = (C.c_char_p * len(frags))(*frags)
    out = C.c_void_p()
    olen = C.c_uint64()
    rc = lib().liberasurecode_decode(desc, arr, len(frags), flen, force, C.byref(out), C.byref(olen))
    data = C.string_at(out.value, olen.value) if rc == 0 and out.value else None
    if rc == 0 and out.value:
        lib().liberasurecode_decode_cleanup(desc, out)
    return rc, data


def reconstruct(desc, frags, flen, dest):
    arr = (C.c_char_p * len(frags))(*frags)
    out = C.create_string_buffer(flen)
    rc = lib().liberasurecode_reconstruct_fragment(desc, arr, len(frags), flen, dest, out)
    return rc, out.raw


def fragments_needed(desc, recon, exclude, n):
    needed = (C.c_int * (n + 1))(*([-1] * (n + 1)))
    r = (C.c_int * (len(recon) + 1))(*(list(recon) + [-1]))
    e = (C.c_int * (len(exclude) + 1))(*(list(exclude) + [-1]))
    rc = lib().liberasurecode_fragments_needed(desc, r, e, needed)
    out = []
    for v in needed:
        if v == -1:
            break
        out.append(v)
    return rc, out


# ---------------------------------------------------------------- framing restatement ----

def crc32_legacy(data: bytes, crc: int = 0) -> int:
    """src/utils/chksum/crc32.c:79-91 restated (sign-extending 8-bit shift)."""
    tab = []
    for n in range(256):
        c = n
        for _ in range(8):
            c = (0xEDB88320 ^ (c >> 1)) if c & 1 else c >> 1
        tab.append(c)
    c = (crc ^ 0xFFFFFFFF) & 0xFFFFFFFF
    for b in data:
        sh = (((c >> 8) & 0xFFFFFF) ^ 0x800000) - 0x800000
        c = (tab[(c ^ b) & 0xFF] ^ sh) & 0xFFFFFFFF
    return c ^ 0xFFFFFFFF


def expected_header(idx, size, orig_size, backend_id, ct, payload: bytes, with_crc=True,
                    legacy=False, chksum_type=None):
    chk = [0] * 8
    ctype = ct if chksum_type is None else chksum_type
    if with_crc and ct == CHKSUM_CRC32:
        chk[0] = crc32_legacy(payload) if legacy else zlib.crc32(payload)
    meta = struct.pack("<IIIQB8IBBI", idx, size, 0, orig_size, ctype, *chk, 0, backend_id,
                       BACKEND_VERSION)
    assert len(meta) == 59
    mcrc = crc32_legacy(meta) if legacy else zlib.crc32(meta)
    return meta + struct.pack("<III", MAGIC, LIBEC_VERSION, mcrc) + b"\0" * 9
