#!/usr/bin/env python3
"""A/B of the late copy in the 16 KiB-tile bitsliced copy-through form (knob bs_late_copy, round 4;
development tool): each input's copy stores after its network and after the next input's loads (the
planes transposed back), so the loads do not wait for the stores.  C5 framed encode without checksum
(32 x 80 MiB objects, k = 20, m = 8, bs = 4 MiB) and the decode-join of data {0..7} (5-8-output
copy-through maps), plus Swift-like (20, 8) objects of 1 MiB (bs = 52432, unaligned chunks: the late copy
does not apply to realigned inputs, a control).  Outputs checked equal; interleaved rounds, median;
fraction of 8 TB/s of the algorithmic bytes."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib, frame  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

VARIANTS = {"early_copy": 0, "late_copy": 1}


def main(rounds=5, reps=6):
    d = _lib.dev()
    d.ecamd_tune(b"bitslice", 2)
    st = D.Stream()
    k, m = 20, 8
    lost = list(range(8))
    for tag, size, S in (("c5", 20 * (4 << 20), 32), ("obj_1MiB_k20", 1 << 20, 2560)):
        fb = frame.FrameBatch(frame.RS_VAND, k, m, size, S, checksum=frame.CHKSUM_NONE)
        obj = D.DeviceBuffer(fb.obj_stride * S)
        _lib.check(d.ecamd_fill_splitmix(obj.ptr, fb.obj_stride, 0, 1, size, S, 0, 0x4E, st.handle), "fill")
        out = D.DeviceBuffer(fb.obj_stride * S)
        bs = fb.blocksize
        ops = {"encode": (lambda: fb.encode(obj, stream=st), S * (size + (k + m) * bs)),
               "decode_join_8": (lambda: fb.decode(lost, out, stream=st), S * (k * bs + size))}
        ref = {}
        for vname, v in VARIANTS.items():
            d.ecamd_tune(b"bs_late_copy", v)
            fb.encode(obj, stream=st)
            st.synchronize()
            frags = fb.fragments()
            fb.decode(lost, out, stream=st)
            st.synchronize()
            joined = out.download()
            if not ref:
                ref = {"f": frags, "j": joined}
            assert (frags == ref["f"]).all() and (joined == ref["j"]).all(), (tag, vname)
        del ref
        times = {}
        a, b = D.Event(), D.Event()
        for _ in range(10):
            ops["encode"][0]()
        for _ in range(rounds):
            for vname, v in VARIANTS.items():
                d.ecamd_tune(b"bs_late_copy", v)
                for op, (fn, _) in ops.items():
                    fn()
                    a.record(st)
                    for _ in range(reps):
                        fn()
                    b.record(st)
                    st.synchronize()
                    times.setdefault((vname, op), []).append(a.elapsed_ms(b) / reps)
        for (vname, op), ts in times.items():
            ms = statistics.median(ts)
            print(json.dumps({"shape": tag, "variant": vname, "op": op, "ms": round(ms, 4),
                              "frac": round(ops[op][1] / (ms * 1e-3) / 8e12, 4)}), flush=True)
        obj.free()
        out.free()
        del fb
    d.ecamd_tune(b"bs_late_copy", -1)
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main()
