#!/usr/bin/env python3
"""One side of an A/B of BitsliceStyle::dpp_reduce (round 4; development tool): the framed CRC32
encode on the bitsliced crc variant, C5 (RS(20,8), 4 MiB payloads, 32 stripes: the fold-each form,
whose per-fragment wave XOR reductions are the ds_bpermute butterfly or DPP + v_readlane) and C3
(RS(10,4), 1 MiB payloads, 256 stripes).  Run once with ECAMD_BS_DPPRED=1 and once without, each with
its own ECAMD_JIT_CACHE; the fragments' sha256 must agree between the runs.  (Since the measurement
dpp_reduce is the default: the baseline side now needs ECAMD_BS_DPPRED=0.)  One JSON line per shape:
median ms and fraction of 8 TB/s of the algorithmic bytes (objects read + payloads written)."""
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
    tag = "bpermute" if os.environ.get("ECAMD_BS_DPPRED") == "0" else "dpp"
    for shape, k, m, size, S in (("c5", 20, 8, 80 << 20, 32), ("c3", 10, 4, 10 << 20, 256)):
        fb = frame.FrameBatch(frame.RS_VAND, k, m, size, S, checksum=frame.CHKSUM_CRC32)
        obj = D.DeviceBuffer(fb.obj_stride * S)
        _lib.check(d.ecamd_fill_splitmix(obj.ptr, fb.obj_stride, 0, 1, size, S, 0, 0x7A, st.handle), "fill")
        fb.encode(obj, stream=st)
        st.synchronize()
        h = hashlib.sha256(fb.fragments().tobytes()).hexdigest()[:16]
        for _ in range(20):
            fb.encode(obj, stream=st)
        a, b = D.Event(), D.Event()
        ts = []
        for _ in range(rounds):
            fb.encode(obj, stream=st)
            a.record(st)
            for _ in range(reps):
                fb.encode(obj, stream=st)
            b.record(st)
            st.synchronize()
            ts.append(a.elapsed_ms(b) / reps)
        ms = statistics.median(ts)
        nbytes = S * (size + (k + m) * fb.blocksize)
        print(json.dumps({"variant": tag, "shape": shape, "ms": round(ms, 4),
                          "frac": round(nbytes / (ms * 1e-3) / 8e12, 4), "frags_sha": h}), flush=True)
        obj.free()
        del fb


if __name__ == "__main__":
    main()
