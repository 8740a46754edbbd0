"""Device-resident framed path (include/ecamd.h, "on-device framing"): S objects in HBM become
S x (k+m) wire-format fragments (80-byte fragment_header_t + payload) byte-identical to the
reference's liberasurecode_encode output, and back (src/erasurecode.c:383-949)."""
import ctypes as C

import numpy as np

from ._lib import check, dev, ints
from .device import DeviceBuffer, _s

RS_VAND = 6       # EC_BACKEND_LIBERASURECODE_RS_VAND
FLAT_XOR_HD = 3   # EC_BACKEND_FLAT_XOR_HD
CHKSUM_NONE = 1
CHKSUM_CRC32 = 2
HEADER = 80


def geometry(backend, k, m, obj_size, hd=3):
    """(blocksize, fragment_len) for an object of obj_size bytes."""
    bs, fl = C.c_int64(), C.c_int64()
    check(dev().ecamd_frame_geometry(backend, k, m, hd, obj_size, C.byref(bs), C.byref(fl)),
          "frame_geometry")
    return bs.value, fl.value


class FrameBatch:
    """S stripes of k+m framed fragments in one device buffer: fragment f of stripe s at
    base + s * stripe_stride + f * frag_stride.

    With `align` = 128 (the default) every payload starts on a 128-byte line: each fragment
    sits in a slot of round_up(80 + blocksize, 128) bytes with its 80-byte header at offset 48
    (base = buffer + 48). Payloads 16 bytes off the line cost the codec 13-19% of its HBM rate
    (tools/pitch_sweep.py); align = 16 packs fragments 16-byte aligned instead."""

    HEADER = 80

    def __init__(self, backend, k, m, obj_size, nstripes, hd=3, checksum=CHKSUM_CRC32, align=128,
                 head=None):
        self.backend, self.k, self.m, self.hd = backend, k, m, hd
        self.checksum = checksum
        self.obj_size = obj_size
        self.nstripes = nstripes
        self.blocksize, self.fragment_len = geometry(backend, k, m, obj_size, hd)
        self.frag_stride = (self.fragment_len + align - 1) // align * align
        self.stripe_stride = self.frag_stride * (k + m)
        # header offset in its slot: payload on an `align` line
        self.head = (-self.HEADER) % align if head is None else head
        # a fragment may run `head` bytes into the next slot (its payload starts the next line)
        self.nbytes = self.stripe_stride * nstripes + self.head
        self.buf = DeviceBuffer(max(self.nbytes, 16))
        self.base = self.buf.ptr + self.head
        self.obj_stride = (obj_size + 15) // 16 * 16

    def encode(self, d_obj: DeviceBuffer, stream=None, obj_stride=None):
        check(dev().ecamd_frame_encode(self.backend, self.k, self.m, self.hd, self.checksum,
                                       d_obj.ptr, obj_stride or self.obj_stride, self.obj_size,
                                       self.base, self.stripe_stride, self.frag_stride,
                                       self.nstripes, _s(stream)), "frame_encode")

    def decode(self, missing, d_obj: DeviceBuffer, stream=None, obj_stride=None):
        check(dev().ecamd_frame_decode(self.backend, self.k, self.m, self.hd,
                                       ints(list(missing) + [-1]), self.base,
                                       self.stripe_stride, self.frag_stride, self.nstripes,
                                       d_obj.ptr, obj_stride or self.obj_stride, self.obj_size,
                                       _s(stream)), "frame_decode")

    def reconstruct(self, missing, dest, stream=None):
        check(dev().ecamd_frame_reconstruct(self.backend, self.k, self.m, self.hd, self.checksum,
                                            ints(list(missing) + [-1]), dest, self.base,
                                            self.stripe_stride, self.frag_stride, self.obj_size,
                                            self.nstripes, _s(stream)), "frame_reconstruct")

    def verify(self, legacy=False, stream=None):
        """(status[S, k+m], crc[S, k+m]) as uint32 arrays (see ecamd_frame_verify)."""
        n = self.nstripes * (self.k + self.m)
        st, crc = DeviceBuffer(max(4 * n, 16)), DeviceBuffer(max(4 * n, 16))
        check(dev().ecamd_frame_verify(self.k + self.m, self.blocksize, int(legacy), self.base,
                                       self.stripe_stride, self.frag_stride, self.nstripes,
                                       st.ptr, crc.ptr, _s(stream)), "frame_verify")
        if stream is not None:
            stream.synchronize()
        shape = (self.nstripes, self.k + self.m)
        return (st.download(4 * n).view(np.uint32).reshape(shape),
                crc.download(4 * n).view(np.uint32).reshape(shape))

    def fragments(self) -> np.ndarray:
        """(S, k+m, fragment_len) uint8 host copy of the wire-format fragments."""
        raw = self.buf.download(self.nbytes)
        return np.ascontiguousarray(self._view(raw))

    def upload_fragments(self, frags: np.ndarray):
        host = np.zeros(self.nbytes, dtype=np.uint8)
        self._view(host)[...] = frags
        self.buf.upload(host)

    def _view(self, flat: np.ndarray) -> np.ndarray:
        """(S, k+m, fragment_len) strided view of the fragments in a flat host image."""
        return np.lib.stride_tricks.as_strided(
            flat[self.head:], shape=(self.nstripes, self.k + self.m, self.fragment_len),
            strides=(self.stripe_stride, self.frag_stride, 1), writeable=True)


def crc32(d_base, nbuf, length, stride, legacy=False, stream=None) -> np.ndarray:
    """zlib crc32 (or the legacy liberasurecode_crc32_alt) of nbuf device buffers of `length`
    bytes at d_base + i * stride."""
    out = DeviceBuffer(max(4 * nbuf, 16))
    check(dev().ecamd_crc32(int(legacy), d_base.ptr if hasattr(d_base, "ptr") else d_base, 0,
                            stride, nbuf, length, 1, out.ptr, _s(stream)), "crc32")
    if stream is not None:
        stream.synchronize()
    return out.download(4 * nbuf).view(np.uint32).copy()
