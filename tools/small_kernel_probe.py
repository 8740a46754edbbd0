#!/usr/bin/env python3
"""Device-only cost of a small RS(10,4) encode (development probe, round 5): `n` ecamd_rs_encode
launches of one stripe with `bs`-byte fragments on device memory, each followed by
hipStreamSynchronize, next to the trivial probe copy kernel; median wall time per launch+wait.  Run
under rocprofv3 --kernel-trace --stats for the kernels' own durations.
usage: small_kernel_probe.py [bs] [n] [knob=value ...]   (knobs: ecamd_tune)"""
import ctypes as C
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from liberasurecode_amd import _lib  # noqa: E402

VP = C.c_void_p


def main():
    bs = int(sys.argv[1]) if len(sys.argv) > 1 else 416
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    hip = C.CDLL("libamdhip64.so.7")  # the runtime torch (imported by _lib) already mapped
    hip.hipStreamSynchronize.argtypes = [VP]
    d = _lib.dev()
    _lib.check(d.ecamd_init(), "init")
    for kv in sys.argv[3:]:
        k, v = kv.split("=")
        _lib.check(d.ecamd_tune(k.encode(), int(v)), kv)
    probe = _lib.probe()
    st = VP()
    assert hip.hipStreamCreate(C.byref(st)) == 0
    buf, other = VP(), VP()
    assert hip.hipMalloc(C.byref(buf), C.c_size_t(max(14 * bs, 1 << 16))) == 0
    assert hip.hipMalloc(C.byref(other), C.c_size_t(1 << 20)) == 0
    assert hip.hipMemset(buf, 7, C.c_size_t(14 * bs)) == 0

    def enc():
        _lib.check(d.ecamd_rs_encode(10, 4, buf, 14 * bs, bs, bs, 1, st), "encode")

    def cp():
        _lib.check(probe.ecamd_probe_copy_tiles(64, other, buf, 4096, st), "copy")

    def launch(mode, nbytes):
        return lambda: _lib.check(probe.ecamd_probe_launch(mode, buf if nbytes else None, nbytes, st), "launch")

    cases = [("rs_encode", enc), ("probe_copy", cp)]
    if os.environ.get("SKP_LAUNCH"):  # the launch probe's fixed-cost kernels (ecamd_probe_launch)
        cases += [("launch_empty", launch(0, 0)), ("launch_stage1_40k", launch(1, 40960)),
                  ("launch_stage8_40k", launch(2, 40960)), ("launch_code32k", launch(4, 0))]
    h = VP()
    assert hip.hipHostMalloc(C.byref(h), C.c_size_t(1 << 16), 0) == 0
    hip.hipMemcpyAsync.argtypes = [VP, VP, C.c_size_t, C.c_int, VP]
    h2d = os.environ.get("SKP_H2D")  # a 4 KiB pinned host -> device copy into the inputs before each launch
    for name, fn in cases + [("rs_encode", enc)]:
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            if h2d:
                assert hip.hipMemcpyAsync(buf, h, 4096, 1, st) == 0
            fn()
            assert hip.hipStreamSynchronize(st) == 0
            ts.append((time.perf_counter() - t0) * 1e6)
        ts = ts[10:]
        print(json.dumps({"case": name, "bs": bs, "median_us": round(statistics.median(ts), 2)}), flush=True)


if __name__ == "__main__":
    main()
