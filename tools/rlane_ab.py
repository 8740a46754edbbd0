#!/usr/bin/env python3
"""One side of an A/B of BitsliceStyle::realign_lane (round 4; development tool): the one-wave
copy-through kernel on Swift's 1 MiB segments (2560 x 1 MiB, bs = 104858: object chunks at unaligned
offsets j*bs, realigned in registers).  Run once with ECAMD_BS_RLANE=1 and once without, each with its
own ECAMD_JIT_CACHE (the request's cache key does not see the experiment flag); the sha256 of the
fragments and of the joined objects must agree between the runs.  Prints one JSON line per op:
median ms and fraction of 8 TB/s of the algorithmic bytes."""
import hashlib
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
    k, m, size, S = 10, 4, 1 << 20, 2560
    tag = "rlane" if os.environ.get("ECAMD_BS_RLANE") == "1" else "base"
    fb = frame.FrameBatch(frame.RS_VAND, k, m, size, S, checksum=frame.CHKSUM_NONE)
    obj = D.DeviceBuffer(fb.obj_stride * S)
    _lib.check(d.ecamd_fill_splitmix(obj.ptr, fb.obj_stride, 0, 1, size, S, 0, 0x7A, st.handle), "fill")
    out = D.DeviceBuffer(fb.obj_stride * S)
    bs = fb.blocksize
    ops = {"encode": (lambda: fb.encode(obj, stream=st), S * (size + (k + m) * bs)),
           "join_0123": (lambda: fb.decode([0, 1, 2, 3], out, stream=st), S * ((k + 4) * bs - 4 * bs + size))}
    fb.encode(obj, stream=st)
    st.synchronize()
    h = hashlib.sha256(fb.fragments().tobytes()).hexdigest()[:16]
    fb.decode([0, 1, 2, 3], out, stream=st)
    st.synchronize()
    hj = hashlib.sha256(out.download().tobytes()).hexdigest()[:16]
    for _ in range(20):
        ops["encode"][0]()
    a, b = D.Event(), D.Event()
    times = {}
    for _ in range(rounds):
        for op, (fn, _) in ops.items():
            fn()
            a.record(st)
            for _ in range(reps):
                fn()
            b.record(st)
            st.synchronize()
            times.setdefault(op, []).append(a.elapsed_ms(b) / reps)
    for op, ts in times.items():
        ms = statistics.median(ts)
        print(json.dumps({"variant": tag, "op": op, "ms": round(ms, 4), "frac": round(ops[op][1] / (ms * 1e-3) / 8e12, 4),
                          "frags_sha": h, "joined_sha": hj}), flush=True)


if __name__ == "__main__":
    main()
