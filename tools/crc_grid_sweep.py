#!/usr/bin/env python3
"""Split CRC32 pass launch shape (development tool): crc_partial_kernel over the C3 payloads (256
stripes x 14 x 1 MiB, random bytes) as a grid-stride loop over 2 / 4 / 8 resident 512-thread
workgroups per CU against one workgroup per 8 spans (crc_wgs huge: the dispatcher hands each freed
slot the next spans), for spans of 16 / 32 / 64 / 128 KiB per wave; interleaved rounds after a
clock-settling warm-up, median, every variant's CRCs checked equal."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib, frame  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

WGS = [int(x) for x in os.environ.get("CRC_WGS", "0,4,8,65536").split(",")]
SPANS = [int(x) for x in os.environ.get("CRC_SPANS", "16,32,64,128").split(",")]


def main(rounds=3, reps=10):
    S, k, m, size = 256, 10, 4, 10 * 1048576
    d = _lib.dev()
    st = D.Stream()
    fb = frame.FrameBatch(frame.RS_VAND, k, m, size, S, align=128)
    _lib.check(d.ecamd_fill_splitmix(fb.base + 80, fb.stripe_stride, fb.frag_stride, k + m,
                                     fb.blocksize, S, 0, 0x5EED, st.handle), "fill")
    crc = D.DeviceBuffer(4 * S * (k + m))
    payload = S * (k + m) * fb.blocksize

    def run():
        _lib.check(d.ecamd_crc32(0, fb.base + 80, fb.stripe_stride, fb.frag_stride, k + m, fb.blocksize, S,
                                 crc.ptr, st.handle), "crc")

    variants = [(w, s) for s in SPANS for w in WGS]
    ref = None
    for w, s in variants:
        d.ecamd_tune(b"crc_wgs", w)
        d.ecamd_tune(b"crc_span_kib", s)
        run()
        st.synchronize()
        got = crc.download(4 * S * (k + m))
        if ref is None:
            ref = got
        assert bool((got == ref).all()), (w, s)
    d.ecamd_tune(b"crc_wgs", 0)
    d.ecamd_tune(b"crc_span_kib", 0)
    for _ in range(60):
        run()
    times = {}
    for _ in range(rounds):
        for w, s in variants:
            d.ecamd_tune(b"crc_wgs", w)
            d.ecamd_tune(b"crc_span_kib", s)
            run()
            a, b = D.Event(), D.Event()
            a.record(st)
            for _ in range(reps):
                run()
            b.record(st)
            st.synchronize()
            times.setdefault((w, s), []).append(a.elapsed_ms(b) / reps)
    for (w, s), ts in times.items():
        med = statistics.median(ts)
        print(json.dumps({"op": "crc32_split", "crc_wgs": w, "span_kib": s, "ms": round(med, 4),
                          "TBps": round(payload / (med * 1e-3) / 1e12, 3),
                          "frac": round(payload / (med * 1e-3) / 8e12, 4)}), flush=True)
    d.ecamd_tune(b"crc_wgs", 0)
    d.ecamd_tune(b"crc_span_kib", 0)


if __name__ == "__main__":
    main()
