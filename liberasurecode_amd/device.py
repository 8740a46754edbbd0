"""Device-resident batched erasure coding on MI355X (Python face of include/ecamd.h).

Buffers are plain HBM allocations made by libecamd (no torch types); a batch of S stripes is a
strided layout where fragment f of stripe s lives at base + s*stripe_stride + f*frag_stride.
"""
import ctypes as C

import numpy as np

from ._lib import check, dev, i64s, ints, u32s


def available() -> bool:
    try:
        return dev().ecamd_init() == 0
    except Exception:
        return False


class DeviceBuffer:
    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        check(dev().ecamd_malloc(C.byref(p), self.nbytes), "ecamd_malloc")
        self.ptr = p.value

    def free(self):
        if self.ptr:
            dev().ecamd_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def upload(self, arr: np.ndarray, offset: int = 0):
        arr = np.ascontiguousarray(arr)
        check(dev().ecamd_memcpy_h2d(self.ptr + offset, arr.ctypes.data, arr.nbytes), "h2d")

    def download(self, nbytes=None, offset: int = 0) -> np.ndarray:
        n = self.nbytes - offset if nbytes is None else int(nbytes)
        out = np.empty(n, dtype=np.uint8)
        check(dev().ecamd_memcpy_d2h(out.ctypes.data, self.ptr + offset, n), "d2h")
        return out

    def zero(self):
        check(dev().ecamd_memset(self.ptr, 0, self.nbytes), "memset")


class Stream:
    def __init__(self):
        p = C.c_void_p()
        check(dev().ecamd_stream_create(C.byref(p)), "stream")
        self.handle = p.value

    def synchronize(self):
        check(dev().ecamd_stream_synchronize(self.handle), "stream sync")

    def destroy(self):
        """ecamd_stream_destroy: the stream and the library's context for it."""
        if self.handle:
            check(dev().ecamd_stream_destroy(self.handle), "stream destroy")
            self.handle = None


class Event:
    def __init__(self):
        p = C.c_void_p()
        check(dev().ecamd_event_create(C.byref(p)), "event")
        self.handle = p.value

    def record(self, stream=None):
        check(dev().ecamd_event_record(self.handle, stream.handle if stream else None), "record")

    def elapsed_ms(self, end: "Event") -> float:
        ms = C.c_float()
        check(dev().ecamd_event_elapsed_ms(self.handle, end.handle, C.byref(ms)), "elapsed")
        return ms.value


def _s(stream):
    return stream.handle if stream is not None else None


class Layout:
    """Strided batch layout of S stripes x F fragments of `blocksize` bytes."""

    def __init__(self, buf: DeviceBuffer, nfrags: int, blocksize: int, nstripes: int,
                 frag_stride=None, stripe_stride=None):
        self.buf = buf
        self.nfrags = nfrags
        self.blocksize = blocksize
        self.nstripes = nstripes
        self.frag_stride = frag_stride or (blocksize + 15) // 16 * 16
        self.stripe_stride = stripe_stride or self.frag_stride * nfrags

    @classmethod
    def alloc(cls, nfrags, blocksize, nstripes):
        fs = (blocksize + 15) // 16 * 16
        buf = DeviceBuffer(fs * nfrags * nstripes)
        return cls(buf, nfrags, blocksize, nstripes, fs, fs * nfrags)

    def upload_stripes(self, frags: np.ndarray):
        """frags: (S, F, blocksize) uint8."""
        S, F, bs = frags.shape
        host = np.zeros((S, self.stripe_stride), dtype=np.uint8)
        for f in range(F):
            host[:, f * self.frag_stride:f * self.frag_stride + bs] = frags[:, f]
        self.buf.upload(host)

    def download_stripes(self) -> np.ndarray:
        raw = self.buf.download(self.stripe_stride * self.nstripes).reshape(self.nstripes,
                                                                             self.stripe_stride)
        out = np.empty((self.nstripes, self.nfrags, self.blocksize), dtype=np.uint8)
        for f in range(self.nfrags):
            out[:, f] = raw[:, f * self.frag_stride:f * self.frag_stride + self.blocksize]
        return out

    def fill_splitmix(self, nfrags=None, stripe0=0, seed_base=0xEC0DE, stream=None):
        check(dev().ecamd_fill_splitmix(self.buf.ptr, self.stripe_stride, self.frag_stride,
                                        nfrags or self.nfrags, self.blocksize, self.nstripes,
                                        stripe0, seed_base, _s(stream)), "fill")


def rs_encode(k, m, lay: Layout, stream=None):
    check(dev().ecamd_rs_encode(k, m, lay.buf.ptr, lay.stripe_stride, lay.frag_stride,
                                lay.blocksize, lay.nstripes, _s(stream)), "rs_encode")


def rs_decode(k, m, missing, lay: Layout, rebuild_parity=True, stream=None):
    check(dev().ecamd_rs_decode(k, m, ints(list(missing) + [-1]), int(rebuild_parity), lay.buf.ptr,
                                lay.stripe_stride, lay.frag_stride, lay.blocksize, lay.nstripes,
                                _s(stream)), "rs_decode")


def rs_decode_multi(k, m, missing_per_stripe, lay: Layout, rebuild_parity=True, stream=None):
    """One erasure list per stripe; stripes are grouped by pattern on the host."""
    width = m + 1
    flat = []
    for pat in missing_per_stripe:
        row = list(pat)[:m] + [-1] * (width - min(len(pat), m))
        flat += row
    check(dev().ecamd_rs_decode_multi(k, m, ints(flat), width, int(rebuild_parity), lay.buf.ptr,
                                      lay.stripe_stride, lay.frag_stride, lay.blocksize,
                                      lay.nstripes, _s(stream)), "rs_decode_multi")


def rs_reconstruct(k, m, missing, dest, lay: Layout, stream=None):
    check(dev().ecamd_rs_reconstruct(k, m, ints(list(missing) + [-1]), dest, lay.buf.ptr,
                                     lay.stripe_stride, lay.frag_stride, lay.blocksize,
                                     lay.nstripes, _s(stream)), "rs_reconstruct")


class GF16Map:
    """An arbitrary R x K GF(2^16) fragment map prepared on the device."""

    def __init__(self, coeff):
        coeff = np.asarray(coeff, dtype=np.int64)
        self.R, self.K = coeff.shape
        p = C.c_void_p()
        check(dev().ecamd_map_create(ints(coeff.reshape(-1).tolist()), self.R, self.K, C.byref(p)),
              "map_create")
        self.handle = p.value

    def __del__(self):
        try:
            dev().ecamd_map_destroy(self.handle)
        except Exception:
            pass

    def apply(self, lay: Layout, inputs, outputs, stream=None, out_layout: Layout = None):
        out_layout = out_layout or lay
        check(dev().ecamd_map_apply_strided(
            self.handle, lay.buf.ptr, lay.stripe_stride,
            i64s([i * lay.frag_stride for i in inputs]), out_layout.buf.ptr,
            out_layout.stripe_stride, i64s([o * out_layout.frag_stride for o in outputs]),
            lay.blocksize, lay.nstripes, _s(stream)), "map_apply")


def xor_encode(k, m, hd, lay: Layout, stream=None):
    """flat_xor_hd encode of a strided batch in place (ecamd_xor_encode)."""
    check(dev().ecamd_xor_encode(k, m, hd, lay.buf.ptr, lay.stripe_stride, lay.frag_stride,
                                 lay.blocksize, lay.nstripes, _s(stream)), "xor_encode")


def xor_decode(k, m, hd, missing, lay: Layout, decode_parity=True, stream=None):
    """xor_hd_decode replayed on every stripe (missing slots read as zero)."""
    check(dev().ecamd_xor_decode(k, m, hd, ints(list(missing) + [-1]), int(decode_parity),
                                 lay.buf.ptr, lay.stripe_stride, lay.frag_stride, lay.blocksize,
                                 lay.nstripes, _s(stream)), "xor_decode")


def xor_reconstruct(k, m, hd, missing, dest, lay: Layout, stream=None):
    """xor_reconstruct_one of fragment `dest` on every stripe."""
    check(dev().ecamd_xor_reconstruct(k, m, hd, ints(list(missing) + [-1]), dest, lay.buf.ptr,
                                      lay.stripe_stride, lay.frag_stride, lay.blocksize,
                                      lay.nstripes, _s(stream)), "xor_reconstruct")


def xor_decode_multi(k, m, hd, missing_per_stripe, lay: Layout, decode_parity=True, stream=None):
    """One erasure list per stripe; stripes with identical lists share a launch."""
    width = k + m + 1
    flat = []
    for pat in missing_per_stripe:
        flat += list(pat)[:width - 1] + [-1] * (width - min(len(pat), width - 1))
    check(dev().ecamd_xor_decode_multi(k, m, hd, ints(flat), width, int(decode_parity), lay.buf.ptr,
                                       lay.stripe_stride, lay.frag_stride, lay.blocksize,
                                       lay.nstripes, _s(stream)), "xor_decode_multi")


def xor_apply(masks, lay: Layout, inputs, outputs, stream=None):
    check(dev().ecamd_xor_apply_strided(
        u32s(masks), len(outputs), len(inputs), lay.buf.ptr, lay.stripe_stride,
        i64s([i * lay.frag_stride for i in inputs]), lay.buf.ptr, lay.stripe_stride,
        i64s([o * lay.frag_stride for o in outputs]), lay.blocksize, lay.nstripes, _s(stream)),
        "xor_apply")


def synchronize():
    check(dev().ecamd_synchronize(), "synchronize")
