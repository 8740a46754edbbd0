#!/usr/bin/env python3
"""A/B of the framed flat-XOR decode with data lost (knob frame_xor_copy, round 4; development tool):
1 = one decode-join launch (the plan's 0 / 1 matrix: lost data straight into the objects, surviving
data copied there), 0 = decode in place + join.  (10,6,4), data {0,1,2} lost, Swift's 1 MiB segments
(2560) and 10 MiB objects (256).  Objects checked equal across the variants first; interleaved rounds,
median; fraction of 8 TB/s of the algorithmic bytes (the k surviving-or-needed payloads read + the
objects written)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib, frame  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

VARIANTS = {"decode_join": 1, "decode_in_place_then_join": 0}


def main(rounds=5, reps=10):
    d = _lib.dev()
    d.ecamd_tune(b"bitslice", 2)
    st = D.Stream()
    k, m, hd, lost = 10, 6, 4, [0, 1, 2]
    for tag, size, S in (("swift_1MiB_segment", 1 << 20, 2560), ("obj_10MiB", 10 << 20, 256)):
        fb = frame.FrameBatch(frame.FLAT_XOR_HD, k, m, size, S, hd=hd)
        obj = D.DeviceBuffer(fb.obj_stride * S)
        _lib.check(d.ecamd_fill_splitmix(obj.ptr, fb.obj_stride, 0, 1, size, S, 0, 0x2D, st.handle), "fill")
        fb.encode(obj, stream=st)
        st.synchronize()
        out = D.DeviceBuffer(fb.obj_stride * S)
        ref = None
        for v in VARIANTS.values():
            d.ecamd_tune(b"frame_xor_copy", v)
            fb.decode(lost, out, stream=st)
            st.synchronize()
            got = out.download()
            if ref is None:
                ref = got
            assert (got == ref).all(), (tag, v)
            del got
        del ref
        algo = S * (size + k * fb.blocksize)
        times = {}
        a, b = D.Event(), D.Event()
        for _ in range(10):
            fb.decode(lost, out, stream=st)
        for _ in range(rounds):
            for vname, v in VARIANTS.items():
                d.ecamd_tune(b"frame_xor_copy", v)
                fb.decode(lost, out, stream=st)
                a.record(st)
                for _ in range(reps):
                    fb.decode(lost, out, stream=st)
                b.record(st)
                st.synchronize()
                times.setdefault(vname, []).append(a.elapsed_ms(b) / reps)
        for vname, ts in times.items():
            ms = statistics.median(ts)
            print(json.dumps({"shape": tag, "variant": vname, "ms": round(ms, 4),
                              "frac": round(algo / (ms * 1e-3) / 8e12, 4)}), flush=True)
        obj.free()
        out.free()
        del fb
    d.ecamd_tune(b"frame_xor_copy", 1)
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main()
