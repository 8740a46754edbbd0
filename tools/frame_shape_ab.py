#!/usr/bin/env python3
"""Framed RS(10,4) encode / systematic join across object sizes (development tool, round 5):

  frame_shape_ab.py size[,size...] [--only op:checksum]   (e.g. --only encode:1, for a profiler run)

Each size gets S = round(2.5 GiB / size) objects; prints the median (3 interleaved rounds of 5) of the
framed encode without checksum, with CRC32, and the systematic join, as the fraction of 8 TB/s of the
algorithmic bytes (objects read + payloads written; payloads read + objects written).  Separates the
cost of small payloads from that of unaligned object chunks (Swift's 1 MiB segments: bs = 104858)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib, frame  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402


def main():
    sizes = [int(v) for v in sys.argv[1].split(",")]
    only = sys.argv[sys.argv.index("--only") + 1].split(":") if "--only" in sys.argv else None
    k, m = 10, 4
    d = _lib.dev()
    d.ecamd_tune(b"bitslice", 2)  # every bitsliced kernel compiled before its first launch
    st = D.Stream()
    cases = {}
    keep = []
    for size in sizes:
        S = max(1, round((5 << 29) / size))
        obj_stride = (size + 15) // 16 * 16
        obj = D.DeviceBuffer(obj_stride * S)
        _lib.check(d.ecamd_fill_splitmix(obj.ptr, obj_stride, 0, 1, size, S, 0, 0x5A, st.handle), "fill")
        out = D.DeviceBuffer(obj_stride * S)
        keep += [obj, out]
        for ct in (frame.CHKSUM_NONE, frame.CHKSUM_CRC32):
            fb = frame.FrameBatch(frame.RS_VAND, k, m, size, S, checksum=ct)
            keep.append(fb)
            bs = fb.blocksize
            cases[(size, S, bs, ct, "encode")] = (lambda fb=fb, obj=obj: fb.encode(obj, stream=st), S * (size + (k + m) * bs))
            if ct == frame.CHKSUM_NONE:
                fb.encode(obj, stream=st)
                cases[(size, S, bs, ct, "join")] = (lambda fb=fb, out=out: fb.decode([], out, stream=st), S * (k * bs + size))
    if only:
        cases = {key: v for key, v in cases.items() if key[4] == only[0] and key[3] == int(only[1])}
    times = {}
    a, b = D.Event(), D.Event()
    for _ in range(3):
        for key, (fn, _) in cases.items():
            fn()
            a.record(st)
            for _ in range(5):
                fn()
            b.record(st)
            st.synchronize()
            times.setdefault(key, []).append(a.elapsed_ms(b) / 5)
    for (size, S, bs, ct, op), ts in times.items():
        ms = statistics.median(ts)
        algo = cases[(size, S, bs, ct, op)][1]
        print(json.dumps({"size": size, "stripes": S, "bs": bs, "checksum": ct, "op": op, "ms": round(ms, 4),
                          "frac": round(algo / (ms * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
