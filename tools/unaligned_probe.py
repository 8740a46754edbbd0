#!/usr/bin/env python3
"""What an unaligned side costs a streaming copy (round 4; development tool, libecamd_probe.so
ecamd_probe_unaligned): 2 GiB copied in one-workgroup 4 KiB tiles with one side displaced by `shift`
bytes -- the object side of the framed copies and of the copy-through codec at offsets j*bs when
bs % 16 != 0 (Swift's 1 MiB segments: bs % 16 = 10, so j*bs % 16 runs over the even shifts).
Modes: aligned, unaligned 16-byte loads, two aligned loads realigned, one aligned load + the next
lane's (DPP), a dword-aligned 16-byte load + one dword, unaligned 16-byte stores.  The copied bytes
are checked for every (mode, shift) first; interleaved rounds, median, fraction of 8 TB/s of
read + written bytes."""
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

MODES = {0: "aligned", 1: "unaligned_b128_load", 2: "two_aligned_loads", 3: "aligned_load_dpp_next",
         4: "dword_aligned_load_plus_dword", 5: "unaligned_b128_store"}
SHIFTS = (0, 2, 4, 8, 10)


def main(rounds=5, reps=10, nbytes=2 << 30):
    p = _lib.probe()
    p.ecamd_probe_unaligned.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
    st = D.Stream()
    src = D.DeviceBuffer(nbytes + 64)
    dst = D.DeviceBuffer(nbytes + 64)
    d = _lib.dev()
    _lib.check(d.ecamd_fill_splitmix(src.ptr, nbytes + 64, 0, 1, nbytes + 64, 1, 0, 0x77, st.handle), "fill")
    st.synchronize()
    # check on a small prefix: 16 tiles
    small = 16 * 4096
    ref = src.download(small + 64)
    for mode in MODES:
        for sh in SHIFTS:
            assert p.ecamd_probe_unaligned(mode, sh, dst.ptr, src.ptr, small, st.handle) == 0
            st.synchronize()
            got = dst.download(small + 64)
            if mode == 0:
                ok = np.array_equal(got[:small], ref[:small])
            elif mode == 5:
                ok = np.array_equal(got[sh:sh + small], ref[:small])
            else:
                ok = np.array_equal(got[:small], ref[sh:sh + small])
            assert ok, (MODES[mode], sh)
    times = {}
    a, b = D.Event(), D.Event()
    for _ in range(rounds):
        for mode in MODES:
            for sh in (SHIFTS if mode else (0,)):
                p.ecamd_probe_unaligned(mode, sh, dst.ptr, src.ptr, nbytes, st.handle)
                a.record(st)
                for _ in range(reps):
                    p.ecamd_probe_unaligned(mode, sh, dst.ptr, src.ptr, nbytes, st.handle)
                b.record(st)
                st.synchronize()
                times.setdefault((mode, sh), []).append(a.elapsed_ms(b) / reps)
    for (mode, sh), ts in times.items():
        ms = statistics.median(ts)
        print(json.dumps({"mode": MODES[mode], "shift": sh, "ms": round(ms, 4),
                          "frac": round(2 * nbytes / (ms * 1e-3) / 8e12, 4)}), flush=True)
    src.free()
    dst.free()


if __name__ == "__main__":
    main()
