#!/usr/bin/env python3
"""Fragment-slot alignment A/B on Swift's 1 MiB EC segments (development tool, round 5):

  frame_align_ab.py [align,...]

FrameBatch(align=A) gives each fragment a slot of round_up(80 + bs, A) bytes (payload on an A-byte
boundary): A changes only where the 14 payload streams sit in HBM, not the bytes moved.  Times the
framed encode (no checksum, CRC32) and the systematic join of 2560 segments (bs = 104858) per
alignment, interleaved rounds, median; fraction of 8 TB/s of the algorithmic bytes.  Every
variant's fragments are checked byte-equal to the first one's (header + payload of each slot)."""
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
    aligns = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "128,1024,4096,16384,65536").split(",")]
    k, m, size, S = 10, 4, 1 << 20, 2560
    d = _lib.dev()
    st = D.Stream()
    obj_stride = (size + 15) // 16 * 16
    obj = D.DeviceBuffer(obj_stride * S)
    _lib.check(d.ecamd_fill_splitmix(obj.ptr, obj_stride, 0, 1, size, S, 0, 0x5A, st.handle), "fill")
    out = D.DeviceBuffer(obj_stride * S)
    cases = {}
    ref = {}
    for a in aligns:
        for ct in (frame.CHKSUM_NONE, frame.CHKSUM_CRC32):
            fb = frame.FrameBatch(frame.RS_VAND, k, m, size, S, checksum=ct, align=a)
            fb.encode(obj, stream=st)
            st.synchronize()
            got = fb.fragments()
            assert (got == ref.setdefault(ct, got)).all(), (a, ct)
            bs = fb.blocksize
            cases[(a, ct, "encode")] = (fb, lambda fb=fb: fb.encode(obj, stream=st), S * (size + (k + m) * bs))
            if ct == frame.CHKSUM_NONE:
                cases[(a, ct, "join")] = (fb, lambda fb=fb: fb.decode([], out, stream=st), S * (k * bs + size))
    times = {}
    ev0, ev1 = D.Event(), D.Event()
    for _ in range(3):
        for key, (fb, fn, _) in cases.items():
            fn()
            ev0.record(st)
            for _ in range(5):
                fn()
            ev1.record(st)
            st.synchronize()
            times.setdefault(key, []).append(ev0.elapsed_ms(ev1) / 5)
    for (a, ct, op), ts in times.items():
        ms = statistics.median(ts)
        algo = cases[(a, ct, op)][2]
        print(json.dumps({"align": a, "frag_stride": cases[(a, ct, op)][0].frag_stride, "checksum": ct, "op": op,
                          "ms": round(ms, 4), "frac": round(algo / (ms * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
