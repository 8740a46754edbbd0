#!/usr/bin/env python3
"""A/B of one knob (ecamd_tune) on the framed device paths (development tool, round 5):

  frame_knob_ab.py KNOB v1,v2,... [--ct crc|none|both] [--ops encode,join,decode]

Shapes: C3 objects (256 x 10 MiB, bs = 1 MiB), Swift's 1 MiB segments (2560 x 1 MiB, bs = 104858)
and C5 objects (32 x 80 MiB, bs = 4 MiB).  Ops: the framed encode (objects read, k + m payloads
written: ecamd_frame_encode), the systematic join (every data payload present: k payloads read,
the object written) and the decode-join of data {0,1,2,3} (4 data lost: k payloads read, the
object written).  Every variant's fragments / objects are checked byte-equal to the first
variant's before timing; interleaved rounds, median; fraction of 8 TB/s of the algorithmic bytes."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib, frame  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

SHAPES = (("c3", 10, 4, 10 << 20, 256), ("swift_1MiB_segment", 10, 4, 1 << 20, 2560), ("c5", 20, 8, 80 << 20, 32))


def main():
    knob = sys.argv[1].encode()
    values = [int(v) for v in sys.argv[2].split(",")]
    ct_arg = sys.argv[sys.argv.index("--ct") + 1] if "--ct" in sys.argv else "both"
    cts = {"crc": [frame.CHKSUM_CRC32], "none": [frame.CHKSUM_NONE],
           "both": [frame.CHKSUM_NONE, frame.CHKSUM_CRC32]}[ct_arg]
    ops_sel = (sys.argv[sys.argv.index("--ops") + 1] if "--ops" in sys.argv else "encode,join,decode").split(",")
    d = _lib.dev()
    d.ecamd_tune(b"bitslice", 2)
    st = D.Stream()
    for tag, k, m, size, S in SHAPES:
        for ct in cts:
            fb = frame.FrameBatch(frame.RS_VAND, k, m, size, S, checksum=ct)
            obj = D.DeviceBuffer(fb.obj_stride * S)
            _lib.check(d.ecamd_fill_splitmix(obj.ptr, fb.obj_stride, 0, 1, size, S, 0, 0x5A, st.handle), "fill")
            out = D.DeviceBuffer(fb.obj_stride * S)
            bs = fb.blocksize
            ops = {"encode": (lambda: fb.encode(obj, stream=st), S * (size + (k + m) * bs)),
                   "join": (lambda: fb.decode([], out, stream=st), S * (k * bs + size)),
                   "decode": (lambda: fb.decode([0, 1, 2, 3], out, stream=st), S * (k * bs + size))}
            ops = {o: v for o, v in ops.items() if o in ops_sel}
            ref = None
            for v in values:
                d.ecamd_tune(knob, v)
                got = []
                for op, (fn, _) in ops.items():
                    if op != "encode":
                        fb.encode(obj, stream=st)
                    fn()
                    st.synchronize()
                    got.append(fb.fragments() if op == "encode" else out.download())
                if ref is None:
                    ref = got
                assert all((a == b).all() for a, b in zip(got, ref)), (tag, ct, v)
            times = {}
            for _ in range(20):
                list(ops.values())[0][0]()
            a, b = D.Event(), D.Event()
            for _ in range(3):
                for v in values:
                    d.ecamd_tune(knob, v)
                    for op, (fn, _) in ops.items():
                        fn()
                        a.record(st)
                        for _ in range(5):
                            fn()
                        b.record(st)
                        st.synchronize()
                        times.setdefault((v, op), []).append(a.elapsed_ms(b) / 5)
            for (v, op), ts in times.items():
                ms = statistics.median(ts)
                print(json.dumps({"shape": tag, "checksum": ct, knob.decode(): v, "op": op, "ms": round(ms, 4),
                                  "frac": round(ops[op][1] / (ms * 1e-3) / 8e12, 4)}), flush=True)
            obj.free()
            out.free()
            del fb
    d.ecamd_tune(knob, -1)
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main()
