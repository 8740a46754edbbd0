"""ctypes view of oracle/build/libec_oracle.so -- the CPU checker (test infrastructure only)."""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
IP = C.POINTER(C.c_int)
_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(os.path.join(ROOT, "oracle", "build", "libec_oracle.so"))
        _lib.orc_gf_mul.argtypes = [C.c_int, C.c_int]
        _lib.orc_gf_inv.argtypes = [C.c_int]
        _lib.orc_gf_table_digest.restype = C.c_uint64
        _lib.orc_rs_generator.argtypes = [C.c_int, C.c_int, IP]
        _lib.orc_gauss_inverse.argtypes = [IP, IP, C.c_int]
        _lib.orc_rs_encode.argtypes = [IP, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int]
        _lib.orc_rs_decode.argtypes = [IP, C.c_void_p, C.c_void_p, C.c_int, C.c_int, IP, C.c_int,
                                       C.c_int]
        _lib.orc_rs_reconstruct.argtypes = [IP, C.c_void_p, C.c_void_p, C.c_int, C.c_int, IP,
                                            C.c_int, C.c_int]
        _lib.orc_gf_init()
    return _lib


def ints(vals):
    return (C.c_int * len(vals))(*vals)


def ptr_array(arrs):
    return (C.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


def generator(k, m):
    out = (C.c_int * ((k + m) * k))()
    assert lib().orc_rs_generator(k, m, out) == 0
    return list(out)


def encode(k, m, data):
    """data: (k, bs) uint8 -> parity (m, bs)."""
    bs = data.shape[1]
    data = np.ascontiguousarray(data)
    par = np.zeros((m, bs), dtype=np.uint8)
    G = ints(generator(k, m))
    lib().orc_rs_encode(G, ptr_array(list(data)), ptr_array(list(par)), k, m, bs)
    return par


def decode(k, m, frags, missing, rebuild_parity=1):
    """frags: list of k+m uint8 arrays (missing ones overwritten in place). Returns rc."""
    bs = frags[0].shape[0]
    G = ints(generator(k, m))
    return lib().orc_rs_decode(G, ptr_array(frags[:k]), ptr_array(frags[k:]), k, m,
                               ints(list(missing) + [-1]), bs, rebuild_parity)


def reconstruct(k, m, frags, missing, dest):
    bs = frags[0].shape[0]
    G = ints(generator(k, m))
    return lib().orc_rs_reconstruct(G, ptr_array(frags[:k]), ptr_array(frags[k:]), k, m,
                                     ints(list(missing) + [-1]), dest, bs)


def crc32(data, legacy=False) -> int:
    """zlib crc32 / liberasurecode_crc32_alt of a bytes-like or uint8 array (oracle restatement)."""
    L = lib()
    fn = L.orc_crc32_alt if legacy else L.orc_crc32
    fn.restype = C.c_uint32
    fn.argtypes = [C.c_uint32, C.c_void_p, C.c_int64]
    buf = np.ascontiguousarray(np.frombuffer(bytes(data), dtype=np.uint8)
                               if not isinstance(data, np.ndarray) else data)
    return fn(0, buf.ctypes.data, buf.size)
