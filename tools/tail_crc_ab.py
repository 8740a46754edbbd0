#!/usr/bin/env python3
"""A/B of the Swift segment CRC32 encode's tail (round 4, development tool): the CRC32 pass's span length
(knob crc_span_kib) and grid, and frame_tail_tiles, on the Swift
segment CRC32 encode (2560 x 1 MiB, bs = 104858), whose serial tail checksums the 6554 bytes past
the 16 KiB tiles of every payload in a run_crc launch of its own (one 8 KiB span per payload by
default: 35840 waves of one span each).  Fragments checked equal; interleaved rounds, median ms."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib, frame  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

# (crc_span_kib, crc_wgs, frame_tail_tiles): round 4 first run -- span / grid of the tail's CRC pass
# (profiles/r04_tail_crc_ab.log: the default best); second -- the whole 4 KiB tile past the 16 KiB
# tiles by the copy-through launch before the split (frame_tail_tiles)
VARIANTS = {"tail_tiles_off": (0, 0, 0), "tail_tiles_on": (0, 0, 1)}


def main(rounds=5, reps=10):
    d = _lib.dev()
    d.ecamd_tune(b"bitslice", 2)
    st = D.Stream()
    k, m, size, S = 10, 4, 1 << 20, 2560
    fb = frame.FrameBatch(frame.RS_VAND, k, m, size, S, checksum=frame.CHKSUM_CRC32)
    obj = D.DeviceBuffer(fb.obj_stride * S)
    _lib.check(d.ecamd_fill_splitmix(obj.ptr, fb.obj_stride, 0, 1, size, S, 0, 0x7A, st.handle), "fill")
    nbytes = S * (size + (k + m) * fb.blocksize)

    def setv(v):
        d.ecamd_tune(b"crc_span_kib", v[0])
        d.ecamd_tune(b"crc_wgs", v[1])
        d.ecamd_tune(b"frame_tail_tiles", v[2])

    ref = None
    for v in VARIANTS.values():
        setv(v)
        fb.encode(obj, stream=st)
        st.synchronize()
        f = fb.fragments()
        if ref is None:
            ref = f
        assert (f == ref).all(), v
    del ref, f
    for _ in range(20):
        fb.encode(obj, stream=st)
    a, b = D.Event(), D.Event()
    times = {}
    for _ in range(rounds):
        for name, v in VARIANTS.items():
            setv(v)
            fb.encode(obj, stream=st)
            a.record(st)
            for _ in range(reps):
                fb.encode(obj, stream=st)
            b.record(st)
            st.synchronize()
            times.setdefault(name, []).append(a.elapsed_ms(b) / reps)
    for name, ts in times.items():
        ms = statistics.median(ts)
        print(json.dumps({"shape": "swift_1MiB_segment_crc32", "variant": name, "ms": round(ms, 4),
                          "frac": round(nbytes / (ms * 1e-3) / 8e12, 4)}), flush=True)
    setv((0, 0, -1))
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main()
