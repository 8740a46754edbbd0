#!/usr/bin/env python3
"""Copy-through framed encode of objects whose payload chunks start at offsets that are not
multiples of 16 (development tool): Swift's 1 MiB segments at k = 10 (bs = 104858, 2560 objects)
and a k = 10 object of 10 MiB + 10 bytes, with the inputs read as aligned chunks realigned in
registers (knob stream_realign 1, gf16_realign_kernel; 2: one aligned load per lane, the second
chunk from the next lane by DPP, round 4) against unaligned 16-byte loads (0);
CHKSUM_NONE and CRC32; interleaved rounds after a clock-settling warm-up, median; fragments
checked equal between the two."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib, frame  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402


def main(rounds=5, reps=5):
    d = _lib.dev()
    st = D.Stream()
    k, m = 10, 4
    for tag, size, S in (("swift_1MiB_segment", 1 << 20, 2560), ("c3_plus_10B", (10 << 20) + 10, 256)):
        fb = frame.FrameBatch(frame.RS_VAND, k, m, size, S)
        obj = D.DeviceBuffer(fb.obj_stride * S)
        _lib.check(d.ecamd_fill_splitmix(obj.ptr, fb.obj_stride, 0, 1, size, S, 0, 0x5A, st.handle), "fill")
        for ct in (frame.CHKSUM_NONE, frame.CHKSUM_CRC32):
            fb.checksum = ct
            got = []
            for ra in (2, 1, 0):
                d.ecamd_tune(b"stream_realign", ra)
                fb.encode(obj, stream=st)
                st.synchronize()
                got.append(fb.fragments())
            assert (got[0] == got[2]).all() and (got[1] == got[2]).all(), (tag, ct)
            del got
            for _ in range(20):
                fb.encode(obj, stream=st)
            times = {2: [], 1: [], 0: []}
            a, b = D.Event(), D.Event()
            for _ in range(rounds):
                for ra in (2, 1, 0):
                    d.ecamd_tune(b"stream_realign", ra)
                    fb.encode(obj, stream=st)
                    a.record(st)
                    for _ in range(reps):
                        fb.encode(obj, stream=st)
                    b.record(st)
                    st.synchronize()
                    times[ra].append(a.elapsed_ms(b) / reps)
            algo = S * (k * fb.blocksize + (k + m) * fb.blocksize)
            for ra, ts in times.items():
                med = statistics.median(ts)
                print(json.dumps({"op": "frame_encode_" + tag, "checksum": ct, "stream_realign": ra,
                                  "blocksize": fb.blocksize, "ms": round(med, 4),
                                  "frac": round(algo / med / 1e6 / 8000, 4)}), flush=True)
        d.ecamd_tune(b"stream_realign", 0)
        obj.free()
        fb.buf.free()


if __name__ == "__main__":
    main()
