"""ctypes bindings to the in-tree native libraries (liberasurecode_amd/lib/*.so).

Loading fails loudly if a library has not been built (`python -c "import __graft_entry__ as g;
g.build()"`); there is no pure-Python or CPU fallback for the codec.

PyTorch is imported first when available: torch wheels carry their own libamdhip64.so (soname
libamdhip64.so.7).  Importing torch before libecamd.so makes the dynamic loader bind libecamd to
that already-loaded runtime instead of mapping a second HIP runtime into the process.
"""
import ctypes as C
import os

try:  # single HIP runtime per process (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the C path
    torch = None

# $LIBERASURECODE_AMD_LIBDIR: another directory of the same built libraries (tests run a copy
# without ecamd_jitc / the shipped jit/ objects there)
LIBDIR = os.environ.get("LIBERASURECODE_AMD_LIBDIR") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")

IP = C.POINTER(C.c_int)
I64P = C.POINTER(C.c_int64)
U32P = C.POINTER(C.c_uint32)
VP = C.c_void_p


def _load(name):
    path = os.path.join(LIBDIR, name)
    if not os.path.exists(path):
        raise ImportError(f"liberasurecode_amd: {path} is not built; run __graft_entry__.build()")
    return C.CDLL(path, mode=C.RTLD_GLOBAL)


def _proto(lib, name, res, args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = args
    return f


_host = None
_dev = None


def host():
    """libecamd_host.so: GF(2^16) math and fragment-map planning (no GPU needed)."""
    global _host
    if _host is None:
        h = _load("libecamd_host.so")
        _proto(h, "ecamd_gf16_mul", C.c_int, [C.c_int, C.c_int])
        _proto(h, "ecamd_gf16_inv", C.c_int, [C.c_int])
        _proto(h, "ecamd_rs_generator", C.c_int, [C.c_int, C.c_int, IP])
        _proto(h, "ecamd_gf16_invert", C.c_int, [IP, IP, C.c_int])
        _proto(h, "ecamd_rs_decode_map", C.c_int, [IP, C.c_int, C.c_int, IP, C.c_int, IP, IP, IP, IP])
        _proto(h, "ecamd_rs_reconstruct_map", C.c_int, [IP, C.c_int, C.c_int, IP, C.c_int, IP, IP, IP])
        _proto(h, "ecamd_bitslice_eval", C.c_int,
               [IP, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, IP])
        _proto(h, "ecamd_bitslice_source", C.c_int64,
               [IP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_char_p, C.c_int64])
        _proto(h, "ecamd_split_tables", C.c_int,
               [IP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p])
        _host = h
    return _host


def dev():
    """libecamd.so: HIP kernels and the device C ABI (include/ecamd.h)."""
    global _dev
    if _dev is None:
        d = _load("libecamd.so")
        _proto(d, "ecamd_init", C.c_int, [])
        _proto(d, "ecamd_device_count", C.c_int, [])
        _proto(d, "ecamd_last_error", C.c_char_p, [])
        _proto(d, "ecamd_tune", C.c_int, [C.c_char_p, C.c_int])
        _proto(d, "ecamd_map_create", C.c_int, [IP, C.c_int, C.c_int, C.POINTER(VP)])
        _proto(d, "ecamd_map_destroy", None, [VP])
        _proto(d, "ecamd_map_apply_strided", C.c_int,
               [VP, VP, C.c_int64, I64P, VP, C.c_int64, I64P, C.c_int64, C.c_int, VP])
        _proto(d, "ecamd_map_apply_ptrs", C.c_int,
               [VP, VP, C.c_int, IP, VP, C.c_int, IP, C.c_int64, C.c_int, VP])
        _proto(d, "ecamd_xor_apply_strided", C.c_int,
               [U32P, C.c_int, C.c_int, VP, C.c_int64, I64P, VP, C.c_int64, I64P, C.c_int64,
                C.c_int, VP])
        _proto(d, "ecamd_xor_apply_ptrs", C.c_int,
               [U32P, C.c_int, C.c_int, VP, C.c_int, IP, VP, C.c_int, IP, C.c_int64, C.c_int, VP])
        _proto(d, "ecamd_rs_encode", C.c_int,
               [C.c_int, C.c_int, VP, C.c_int64, C.c_int64, C.c_int64, C.c_int, VP])
        _proto(d, "ecamd_rs_decode", C.c_int,
               [C.c_int, C.c_int, IP, C.c_int, VP, C.c_int64, C.c_int64, C.c_int64, C.c_int, VP])
        _proto(d, "ecamd_rs_decode_multi", C.c_int,
               [C.c_int, C.c_int, IP, C.c_int, C.c_int, VP, C.c_int64, C.c_int64, C.c_int64,
                C.c_int, VP])
        _proto(d, "ecamd_rs_reconstruct", C.c_int,
               [C.c_int, C.c_int, IP, C.c_int, VP, C.c_int64, C.c_int64, C.c_int64, C.c_int, VP])
        _proto(d, "ecamd_xor_encode", C.c_int,
               [C.c_int, C.c_int, C.c_int, VP, C.c_int64, C.c_int64, C.c_int64, C.c_int, VP])
        _proto(d, "ecamd_xor_decode", C.c_int,
               [C.c_int, C.c_int, C.c_int, IP, C.c_int, VP, C.c_int64, C.c_int64, C.c_int64,
                C.c_int, VP])
        _proto(d, "ecamd_xor_reconstruct", C.c_int,
               [C.c_int, C.c_int, C.c_int, IP, C.c_int, VP, C.c_int64, C.c_int64, C.c_int64,
                C.c_int, VP])
        _proto(d, "ecamd_xor_decode_multi", C.c_int,
               [C.c_int, C.c_int, C.c_int, IP, C.c_int, C.c_int, VP, C.c_int64, C.c_int64,
                C.c_int64, C.c_int, VP])
        _proto(d, "ecamd_fill_splitmix", C.c_int,
               [VP, C.c_int64, C.c_int64, C.c_int, C.c_int64, C.c_int, C.c_int, C.c_uint64, VP])
        _proto(d, "ecamd_frame_geometry", C.c_int,
               [C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64, I64P, I64P])
        _proto(d, "ecamd_frame_encode", C.c_int,
               [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, VP, C.c_int64, C.c_uint64, VP,
                C.c_int64, C.c_int64, C.c_int, VP])
        _proto(d, "ecamd_frame_decode", C.c_int,
               [C.c_int, C.c_int, C.c_int, C.c_int, IP, VP, C.c_int64, C.c_int64, C.c_int, VP,
                C.c_int64, C.c_uint64, VP])
        _proto(d, "ecamd_frame_reconstruct", C.c_int,
               [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, IP, C.c_int, VP, C.c_int64,
                C.c_int64, C.c_uint64, C.c_int, VP])
        _proto(d, "ecamd_frame_verify", C.c_int,
               [C.c_int, C.c_int64, C.c_int, VP, C.c_int64, C.c_int64, C.c_int, VP, VP, VP])
        _proto(d, "ecamd_crc32", C.c_int,
               [C.c_int, VP, C.c_int64, C.c_int64, C.c_int, C.c_int64, C.c_int, VP, VP])
        _proto(d, "ecamd_host_map_apply", C.c_int, [IP, C.c_int, C.c_int, VP, VP, C.c_int64])
        _proto(d, "ecamd_percall_crc_arm", C.c_int, [C.c_int])
        _proto(d, "ecamd_percall_crc_lookup", C.c_int, [VP, C.c_int64, C.POINTER(C.c_uint32)])
        _proto(d, "ecamd_percall_crc_disarm", None, [])
        _proto(d, "ecamd_bitslice_available", C.c_int, [])
        _proto(d, "ecamd_bitslice_wait", C.c_int, [])
        _proto(d, "ecamd_bitslice_entries", C.c_int, [])
        _proto(d, "ecamd_bitslice_launches", C.c_longlong, [])
        _proto(d, "ecamd_rs_kernel_form", C.c_int, [C.c_int, C.c_int, VP, C.c_int, C.c_int, C.c_int64])
        _proto(d, "ecamd_bitslice_prebuild", C.c_int,
               [C.c_int, C.c_int, VP, C.c_int, C.c_int, C.c_char_p, C.c_char_p])
        _proto(d, "ecamd_frame_prebuild", C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_char_p, C.c_char_p])
        _proto(d, "ecamd_percall_reset", None, [])
        _proto(d, "ecamd_percall_status", C.c_int, [])
        _proto(d, "ecamd_fault_inject", C.c_int, [C.c_char_p, C.c_int])
        _proto(d, "ecamd_malloc", C.c_int, [C.POINTER(VP), C.c_int64])
        _proto(d, "ecamd_free", C.c_int, [VP])
        _proto(d, "ecamd_memcpy_h2d", C.c_int, [VP, VP, C.c_int64])
        _proto(d, "ecamd_memcpy_d2h", C.c_int, [VP, VP, C.c_int64])
        _proto(d, "ecamd_memset", C.c_int, [VP, C.c_int, C.c_int64])
        _proto(d, "ecamd_memcpy_async", C.c_int, [VP, VP, C.c_int64, C.c_int, VP])
        _proto(d, "ecamd_host_alloc", C.c_int, [C.POINTER(VP), C.c_int64])
        _proto(d, "ecamd_host_free", C.c_int, [VP])
        _proto(d, "ecamd_synchronize", C.c_int, [])
        _proto(d, "ecamd_stream_create", C.c_int, [C.POINTER(VP)])
        _proto(d, "ecamd_stream_destroy", C.c_int, [VP])
        _proto(d, "ecamd_stream_contexts", C.c_int, [])
        _proto(d, "ecamd_stream_synchronize", C.c_int, [VP])
        _proto(d, "ecamd_event_create", C.c_int, [C.POINTER(VP)])
        _proto(d, "ecamd_event_destroy", C.c_int, [VP])
        _proto(d, "ecamd_event_record", C.c_int, [VP, VP])
        _proto(d, "ecamd_event_elapsed_ms", C.c_int, [VP, VP, C.POINTER(C.c_float)])
        _dev = d
    return _dev


_probe = None


def probe():
    """libecamd_probe.so: HBM / lookup-engine measurement probes (not the codec product)."""
    global _probe
    if _probe is None:
        dev()  # same HIP runtime, device selection and memory helpers
        p = _load("libecamd_probe.so")
        _proto(p, "ecamd_probe_last_error", C.c_char_p, [])
        _proto(p, "ecamd_probe_stream_copy", C.c_int, [VP, VP, C.c_int64, VP])
        _proto(p, "ecamd_probe_bw", C.c_int,
               [C.c_int, C.c_int, C.c_int, VP, VP, C.c_int64, VP])
        _proto(p, "ecamd_probe_copy_tiles", C.c_int, [C.c_int, VP, VP, C.c_int64, VP])
        _proto(p, "ecamd_probe_launch", C.c_int, [C.c_int, VP, C.c_int, VP])
        _proto(p, "ecamd_probe_lookup", C.c_int, [C.c_int, C.c_int, C.c_int, VP, VP])
        _proto(p, "ecamd_probe_mix", C.c_int,
               [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, VP, C.c_int64, C.c_int, C.c_int,
                C.c_int, VP])
        _proto(p, "ecamd_probe_mix2", C.c_int,
               [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, VP, C.c_int64,
                C.c_int, C.c_int, C.c_int, VP])
        _proto(p, "ecamd_probe_mix3", C.c_int,
               [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, VP, C.c_int64, C.c_int,
                C.c_int, C.c_int, IP, VP])
        _proto(p, "ecamd_probe_mix4", C.c_int,
               [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, VP, C.c_int64, C.c_int,
                C.c_int, C.c_int, IP, VP])
        _proto(p, "ecamd_probe_valu", C.c_int, [C.c_int, C.c_int, C.c_int, VP])
        _proto(p, "ecamd_probe_mailbox", C.c_int, [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double)])
        _probe = p
    return _probe


class ECAmdError(RuntimeError):
    pass


def check(rc, what=""):
    if rc != 0:
        msg = dev().ecamd_last_error().decode(errors="replace") if _dev is not None else ""
        raise ECAmdError(f"{what} failed ({rc}): {msg}")
    return rc


def ints(vals):
    vals = list(vals)
    return (C.c_int * max(len(vals), 1))(*vals)


def i64s(vals):
    vals = list(vals)
    return (C.c_int64 * max(len(vals), 1))(*vals)


def u32s(vals):
    vals = list(vals)
    return (C.c_uint32 * max(len(vals), 1))(*vals)
