#!/usr/bin/env python3
"""A/B of the bitsliced crc variant's piece tables (round 3): byte tables (16 lookups per 16-byte
piece into 256-entry tables, ~3.5-way LDS bank conflicts) against nibble tables (knob
frame_crc_bs_nib: 32 lookups into 16-entry tables, conflict-free, an image an eighth the size) for the
CHKSUM_CRC32 framed encode at C3 (256 x 10 MiB objects, k=10 m=4) and C5 (32 x 80 MiB, k=20 m=8), with
1 / 2 / 4 position sets.  Fragments of every variant checked equal to the default's; interleaved
rounds, median; fraction of 8 TB/s of the algorithmic bytes (objects read + payloads written)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib, frame  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

SHAPES = [("c3", 10, 4, 1 << 20, 256), ("c5", 20, 8, 4 << 20, 32)]
# (nib, position sets; 0 = by shape: 1 for <= 4 outputs, 2 for 5-8)
VARIANTS = [(0, 0), (1, 0), (1, 1), (1, 2), (1, 4)]


def main(rounds=5, reps=5):
    d = _lib.dev()
    st = D.Stream()
    d.ecamd_tune(b"bitslice", 2)
    for name, k, m, F, S in SHAPES:
        size = k * F
        fb = frame.FrameBatch(frame.RS_VAND, k, m, size, S, checksum=frame.CHKSUM_CRC32)
        obj = D.DeviceBuffer(fb.obj_stride * S)
        _lib.check(d.ecamd_fill_splitmix(obj.ptr, fb.obj_stride, 0, 1, size, S, 0, 0xC3, st.handle), "fill")
        ref = None
        for nib, pos in VARIANTS:  # compile every variant, check its bytes
            d.ecamd_tune(b"frame_crc_bs_nib", nib)
            d.ecamd_tune(b"frame_crc_pos", pos)
            fb.encode(obj, stream=st)
            st.synchronize()
            fr = fb.fragments()
            if ref is None:
                ref = fr
            assert (fr == ref).all(), (name, nib, pos)
            del fr
        del ref
        algo = S * (k + k + m) * F
        times = {v: [] for v in VARIANTS}
        a, b = D.Event(), D.Event()
        for _ in range(20):
            fb.encode(obj, stream=st)
        for _ in range(rounds):
            for nib, pos in VARIANTS:
                d.ecamd_tune(b"frame_crc_bs_nib", nib)
                d.ecamd_tune(b"frame_crc_pos", pos)
                for _ in range(3):
                    fb.encode(obj, stream=st)
                a.record(st)
                for _ in range(reps):
                    fb.encode(obj, stream=st)
                b.record(st)
                st.synchronize()
                times[(nib, pos)].append(a.elapsed_ms(b) / reps)
        for (nib, pos), ts in times.items():
            ms = statistics.median(ts)
            print(json.dumps({"shape": name, "nibble_tables": nib, "crc_pos": pos, "ms": round(ms, 4),
                              "frac": round(algo / (ms * 1e-3) / 8e12, 4)}), flush=True)
        obj.free()
        del fb
    d.ecamd_tune(b"frame_crc_bs_nib", -1)
    d.ecamd_tune(b"frame_crc_pos", -1)
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main()
