#!/usr/bin/env python3
"""Swift-segment framed encode for rocprofv3 (tools/gpu_prof_swift.sh; development tool): 2560 x 1 MiB
objects at k = 10, m = 4 (bs = 104858), 25 encodes after 5 warm-ups, with CRC32 (SWIFT_CHKSUM=2,
the partly fused cover path: crc variant + tail codec + tail CRC + finalize) or without (1: the
copy-through codec).  The kernel trace then shows what each launch of one encode costs."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib, frame  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402


def main(n=25, warm=5):
    ct = int(os.environ.get("SWIFT_CHKSUM", "2"))
    d = _lib.dev()
    d.ecamd_tune(b"bitslice", 2)
    st = D.Stream()
    k, m, size, S = 10, 4, 1 << 20, 2560
    fb = frame.FrameBatch(frame.RS_VAND, k, m, size, S, checksum=ct)
    obj = D.DeviceBuffer(fb.obj_stride * S)
    _lib.check(d.ecamd_fill_splitmix(obj.ptr, fb.obj_stride, 0, 1, size, S, 0, 0x3C, st.handle), "fill")
    for _ in range(warm):
        fb.encode(obj, stream=st)
    a, b = D.Event(), D.Event()
    a.record(st)
    for _ in range(n):
        fb.encode(obj, stream=st)
    b.record(st)
    st.synchronize()
    ms = a.elapsed_ms(b) / n
    algo = S * (size + (k + m) * fb.blocksize)
    print(json.dumps({"op": "swift_encode", "checksum": ct, "ms": round(ms, 4),
                      "frac": round(algo / (ms * 1e-3) / 8e12, 4)}), flush=True)
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main()
