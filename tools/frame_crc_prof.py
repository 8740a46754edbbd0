#!/usr/bin/env python3
"""Framed CHKSUM_CRC32 encode at the C3 shape (256 x 10 MiB objects, RS(10,4)) for rocprofv3
(tools/gpu_prof_frame_crc.sh): the bitsliced crc variant (knob bitslice 2: compiled before the
timed launches), 5 warm-up then `reps` encodes, and the same on the LDS-table fused kernel
(frame_crc_bs 0) after it.  Prints one JSON line per kernel path with the HIP-event time per encode
and the algorithmic bytes (10 MiB read + 14 MiB written per stripe).  Paths (argv, default
bitsliced_crc lds_fused): bitsliced_crc (16 KiB tiles), wave_crc (one-wave 4 KiB tiles, the default
form: knob frame_crc_wave), lds_fused."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib, frame  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402


PATHS = {"bitsliced_crc": {"frame_crc_bs": 1, "frame_crc_wave": 0},
         "wave_crc": {"frame_crc_bs": 1, "frame_crc_wave": -1},  # the default form
         "lds_fused": {"frame_crc_bs": 0, "frame_crc_wave": 0}}


def main(paths, reps=20):
    d = _lib.dev()
    S, k, m, size = 256, 10, 4, 10 << 20
    st = D.Stream()
    fb = frame.FrameBatch(frame.RS_VAND, k, m, size, S, checksum=frame.CHKSUM_CRC32)
    obj = D.DeviceBuffer(fb.obj_stride * S)
    _lib.check(d.ecamd_fill_splitmix(obj.ptr, fb.obj_stride, 0, 1, size, S, 0, 0xF00D, st.handle), "fill")
    algo = S * (k * (1 << 20) + (k + m) * fb.blocksize)
    d.ecamd_tune(b"bitslice", 2)
    for path in paths:
        for kn, v in PATHS[path].items():
            d.ecamd_tune(kn.encode(), v)
        for _ in range(5):
            fb.encode(obj, stream=st)
        a, b = D.Event(), D.Event()
        a.record(st)
        for _ in range(reps):
            fb.encode(obj, stream=st)
        b.record(st)
        st.synchronize()
        ms = a.elapsed_ms(b) / reps
        print(json.dumps({"path": path, "ms_per_encode": round(ms, 4), "algorithmic_bytes": algo,
                          "frac": round(algo / ms / 1e6 / 8000, 4)}), flush=True)
    d.ecamd_tune(b"frame_crc_bs", -1)
    d.ecamd_tune(b"frame_crc_wave", -1)
    d.ecamd_tune(b"bitslice", 1)


if __name__ == "__main__":
    main(sys.argv[1:] or ["bitsliced_crc", "lds_fused"])
