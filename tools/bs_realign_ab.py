#!/usr/bin/env python3
"""A/B of knob bs_realign on the one-wave bitsliced copy-through encode of Swift's 1 MiB segments
(round 4; development tool): 1 = aligned loads realigned in registers (DPP + v_alignbyte, VALU),
0 = unaligned 16-byte buffer loads (no VALU; -3% in a plain copy, profiles/r04_unaligned_probe.log), with
bs_wave_copy 1 (the default) so the one-wave kernel takes the unaligned encode either way.
Fragments checked equal; interleaved rounds, median ms and fraction of 8 TB/s of the algorithmic
bytes (objects read + payloads written)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib, frame  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402


def main(rounds=5, reps=10):
    d = _lib.dev()
    d.ecamd_tune(b"bitslice", 2)
    st = D.Stream()
    k, m = 10, 4
    for tag, size, S in (("swift_1MiB_segment", 1 << 20, 2560), ("c3_plus_10B", (10 << 20) + 10, 256)):
        for ck in (frame.CHKSUM_NONE, frame.CHKSUM_CRC32):
            fb = frame.FrameBatch(frame.RS_VAND, k, m, size, S, checksum=ck)
            obj = D.DeviceBuffer(fb.obj_stride * S)
            _lib.check(d.ecamd_fill_splitmix(obj.ptr, fb.obj_stride, 0, 1, size, S, 0, 0x7A, st.handle), "fill")
            nbytes = S * (size + (k + m) * fb.blocksize)
            ref = None
            for v in (1, 0):
                d.ecamd_tune(b"bs_realign", v)
                d.ecamd_tune(b"bs_wave_copy", 1)
                fb.encode(obj, stream=st)
                st.synchronize()
                f = fb.fragments()
                if ref is None:
                    ref = f
                assert (f == ref).all(), (tag, v)
            del ref, f
            for _ in range(20):
                fb.encode(obj, stream=st)
            a, b = D.Event(), D.Event()
            times = {}
            for _ in range(rounds):
                for v in (1, 0):
                    d.ecamd_tune(b"bs_realign", v)
                    d.ecamd_tune(b"bs_wave_copy", 1)
                    fb.encode(obj, stream=st)
                    a.record(st)
                    for _ in range(reps):
                        fb.encode(obj, stream=st)
                    b.record(st)
                    st.synchronize()
                    times.setdefault(v, []).append(a.elapsed_ms(b) / reps)
            for v, ts in times.items():
                ms = statistics.median(ts)
                print(json.dumps({"shape": tag, "checksum": ck, "bs_realign": v, "ms": round(ms, 4),
                                  "frac": round(nbytes / (ms * 1e-3) / 8e12, 4)}), flush=True)
            obj.free()
            del fb
    d.ecamd_tune(b"bs_realign", -1)
    d.ecamd_tune(b"bs_wave_copy", -1)
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main()
