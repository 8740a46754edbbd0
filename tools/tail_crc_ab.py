#!/usr/bin/env python3
"""A/B of the CRC32 pass's span length (knob crc_span_kib; round 4, development tool) on the Swift
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

VARIANTS = {"auto": (0, 0), "span4": (4, 0), "span4_wgs16": (4, 16), "auto_wgs16": (0, 16)}


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
    setv((0, 0))
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main()
