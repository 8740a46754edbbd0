#!/usr/bin/env python3
"""A/B of the bitsliced crc variant with the next input's loads issued before the current input's copy
stores (knob frame_crc_prefetch 0 / 2 / 4, round 4; development tool): CHKSUM_CRC32 framed encode of
C3 objects (256 x 10 MiB, bs = 1 MiB, the fused launch over whole payloads) and Swift's 1 MiB segments
(2560, bs = 104858: the crc variant over the whole tiles + tails).  Fragments checked equal across the
variants first; interleaved rounds, median; fraction of 8 TB/s of objects read + payloads written."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib, frame  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

VARIANTS = {"pf0": 0, "pf2": 2, "pf4": 4}


def main(rounds=5, reps=10):
    d = _lib.dev()
    d.ecamd_tune(b"bitslice", 2)
    st = D.Stream()
    k, m = 10, 4
    for tag, size, S in (("c3", 10 << 20, 256), ("swift_1MiB_segment", 1 << 20, 2560)):
        fb = frame.FrameBatch(frame.RS_VAND, k, m, size, S, checksum=frame.CHKSUM_CRC32)
        obj = D.DeviceBuffer(fb.obj_stride * S)
        _lib.check(d.ecamd_fill_splitmix(obj.ptr, fb.obj_stride, 0, 1, size, S, 0, 0x51, st.handle), "fill")
        ref = None
        for v in VARIANTS.values():
            d.ecamd_tune(b"frame_crc_prefetch", v)
            fb.encode(obj, stream=st)
            st.synchronize()
            got = fb.fragments()
            if ref is None:
                ref = got
            assert (got == ref).all(), (tag, v)
            del got
        del ref
        algo = S * (size + (k + m) * fb.blocksize)
        for _ in range(20):
            fb.encode(obj, stream=st)
        times = {}
        a, b = D.Event(), D.Event()
        for _ in range(rounds):
            for vname, v in VARIANTS.items():
                d.ecamd_tune(b"frame_crc_prefetch", v)
                fb.encode(obj, stream=st)
                a.record(st)
                for _ in range(reps):
                    fb.encode(obj, stream=st)
                b.record(st)
                st.synchronize()
                times.setdefault(vname, []).append(a.elapsed_ms(b) / reps)
        for vname, ts in times.items():
            ms = statistics.median(ts)
            print(json.dumps({"shape": tag, "variant": vname, "ms": round(ms, 4),
                              "frac": round(algo / (ms * 1e-3) / 8e12, 4)}), flush=True)
        obj.free()
        del fb
    d.ecamd_tune(b"frame_crc_prefetch", 0)
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main()
