#!/usr/bin/env python3
"""Systematic framed decode workload for rocprofv3 (tools/gpu_prof_join.sh): fragments_to_string
only (every data fragment present, src/erasurecode.c:597-607) on the streaming join kernel, 5
warm-up + 20 decodes of 256 C3 objects (10 MiB, bs = 1 MiB), then 5 + 20 of 2560 Swift 1 MiB
segments (k = 10: bs = 104858). Both move 2560 MiB of object bytes per launch (read + write =
5368709120 algorithmic bytes): frame_join_stream_kernel dispatches 5..24 and 30..49 are the
steady windows. Prints the HIP-event rate of each window too."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import frame  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402


def main(warm=5, reps=20):
    st = D.Stream()
    for tag, size, S in (("c3", 10 << 20, 256), ("swift_1MiB_segment", 1 << 20, 2560)):
        fb = frame.FrameBatch(frame.RS_VAND, 10, 4, size, S)
        obj = D.DeviceBuffer(fb.obj_stride * S)
        obj.zero()
        fb.encode(obj, stream=st)
        out = D.DeviceBuffer(fb.obj_stride * S)
        for _ in range(warm):
            fb.decode([], out, stream=st)
        a, b = D.Event(), D.Event()
        a.record(st)
        for _ in range(reps):
            fb.decode([], out, stream=st)
        b.record(st)
        st.synchronize()
        ms = a.elapsed_ms(b) / reps
        algo = 2 * S * size
        print(json.dumps({"op": "frame_decode_systematic_" + tag, "ms": round(ms, 4), "algorithmic_bytes": algo,
                          "frac": round(algo / ms / 1e6 / 8000, 4)}), flush=True)
        obj.free()
        out.free()
        del fb


if __name__ == "__main__":
    main()
