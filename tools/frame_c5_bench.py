#!/usr/bin/env python3
"""Framed C5 (k=20 m=8, 4 MiB payloads, 32 stripes of 80 MiB objects): encode (copy-through,
no checksum) and decode-join of 8 lost fragments ({0..7} and the survey's mixed pattern), on the
bitsliced kernel (knob bitslice 2) against the LDS-table kernels (knob 0), interleaved rounds,
median.  Algorithmic bytes: encode 20 read + 28 written payloads per stripe; decode-join 20 read
(+ the surviving data copied into the objects) + 8 rebuilt, i.e. 20 reads + 20 writes."""
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
    k, m, S = 20, 8, 32
    size = k * (4 << 20)
    st = D.Stream()
    fb = frame.FrameBatch(frame.RS_VAND, k, m, size, S, checksum=frame.CHKSUM_NONE)
    obj = D.DeviceBuffer(fb.obj_stride * S)
    _lib.check(d.ecamd_fill_splitmix(obj.ptr, fb.obj_stride, 0, 1, size, S, 0, 0xC5, st.handle), "fill")
    out = D.DeviceBuffer(fb.obj_stride * S)
    F = 4 << 20
    ops = {
        "encode": (lambda: fb.encode(obj, stream=st), S * (k + k + m) * F),
        "decode_join_0_7": (lambda: fb.decode(list(range(8)), out, stream=st), S * (k + k) * F),
        "decode_join_mixed": (lambda: fb.decode([0, 2, 4, 6, 20, 22, 24, 26], out, stream=st), S * (k + k) * F),
    }
    d.ecamd_tune(b"bitslice", 2)
    for name, (fn, _) in ops.items():  # compile every matrix first
        fn()
    st.synchronize()
    times = {(n, mode): [] for n in ops for mode in (2, 0)}
    a, b = D.Event(), D.Event()
    for _ in range(rounds):
        for mode in (2, 0):
            d.ecamd_tune(b"bitslice", mode)
            for name, (fn, _) in ops.items():
                for _ in range(3):
                    fn()
                a.record(st)
                for _ in range(reps):
                    fn()
                b.record(st)
                st.synchronize()
                times[(name, mode)].append(a.elapsed_ms(b) / reps)
    # CHKSUM_CRC32: the bitsliced crc variant (fold-each form for 8 outputs) against the bitsliced
    # copy-through encode + the split CRC pass (knob frame_crc_bs 0); fragments checked equal
    d.ecamd_tune(b"bitslice", 2)
    fc = frame.FrameBatch(frame.RS_VAND, k, m, size, S, checksum=frame.CHKSUM_CRC32)
    frags = []
    for knob in (1, 0):
        d.ecamd_tune(b"frame_crc_bs", knob)
        fc.encode(obj, stream=st)
        st.synchronize()
        frags.append(fc.fragments())
    assert (frags[0] == frags[1]).all(), "fused and split CRC framing differ"
    del frags
    for _ in range(rounds):
        for knob in (1, 0):
            d.ecamd_tune(b"frame_crc_bs", knob)
            for _ in range(3):
                fc.encode(obj, stream=st)
            a.record(st)
            for _ in range(reps):
                fc.encode(obj, stream=st)
            b.record(st)
            st.synchronize()
            times.setdefault(("encode_crc32", 3 if knob else 4), []).append(a.elapsed_ms(b) / reps)
    ops["encode_crc32"] = (None, S * (k + k + m) * F)
    d.ecamd_tune(b"frame_crc_bs", -1)
    d.ecamd_tune(b"bitslice", 1)
    kernel = {2: "bitsliced", 0: "lds_tables", 3: "bitsliced_crc_variant", 4: "bitsliced_then_split_crc"}
    for (name, mode), ts in times.items():
        med = statistics.median(ts)
        algo = ops[name][1]
        print(json.dumps({"op": "frame_c5_" + name, "kernel": kernel[mode],
                          "ms": round(med, 4), "algorithmic_bytes": algo,
                          "frac": round(algo / med / 1e6 / 8000, 4),
                          "GiBps_object": round(S * size / (med / 1e3) / 2**30, 1)}), flush=True)


if __name__ == "__main__":
    main()
