#!/usr/bin/env python3
"""Where a small per-call request's fixed cost goes (development probe, round 5): median over 300
rounds, one stream, no torch.  A tiny kernel (libecamd_probe copy of 4 KiB) + hipStreamSynchronize;
the same waited by spinning on hipStreamQuery; a 4 KiB pinned H2D copy + sync; copy + kernel + sync;
and the codec's own smallest call through the per-call API is in tools/latency_bench.py."""
import ctypes as C
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
hip = C.CDLL("/opt/rocm/lib/libamdhip64.so")
probe = C.CDLL(os.path.join(ROOT, "liberasurecode_amd", "lib", "libecamd_probe.so"))
VP = C.c_void_p


def chk(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: {rc}")


def main():
    st = VP()
    chk(hip.hipStreamCreate(C.byref(st)), "stream")
    d_a, d_b, h = VP(), VP(), VP()
    chk(hip.hipMalloc(C.byref(d_a), C.c_size_t(1 << 20)), "malloc")
    chk(hip.hipMalloc(C.byref(d_b), C.c_size_t(1 << 20)), "malloc")
    chk(hip.hipHostMalloc(C.byref(h), C.c_size_t(1 << 20), 0), "hostmalloc")
    probe.ecamd_probe_copy_tiles.argtypes = [C.c_int, VP, VP, C.c_int64, VP]
    hip.hipMemcpyAsync.argtypes = [VP, VP, C.c_size_t, C.c_int, VP]
    hip.hipStreamSynchronize.argtypes = [VP]
    hip.hipStreamQuery.argtypes = [VP]

    def kern():
        chk(probe.ecamd_probe_copy_tiles(64, d_b, d_a, 4096, st), "kernel")

    def h2d():
        chk(hip.hipMemcpyAsync(d_a, h, 4096, 1, st), "h2d")

    def sync():
        chk(hip.hipStreamSynchronize(st), "sync")

    def spin():
        while hip.hipStreamQuery(st) != 0:
            pass

    cases = {"kernel+sync": (kern, sync), "kernel+spin": (kern, spin), "h2d+sync": (h2d, sync),
             "h2d+kernel+sync": (lambda: (h2d(), kern()), sync), "h2d+kernel+spin": (lambda: (h2d(), kern()), spin)}
    res = {}
    for _ in range(3):
        for name, (issue, wait) in cases.items():
            ts = []
            for _ in range(100):
                t0 = time.perf_counter()
                issue()
                wait()
                ts.append((time.perf_counter() - t0) * 1e6)
            res.setdefault(name, []).extend(ts[10:])
    for name, ts in res.items():
        print(json.dumps({"case": name, "median_us": round(statistics.median(ts), 2),
                          "p10_us": round(sorted(ts)[len(ts) // 10], 2)}), flush=True)


if __name__ == "__main__":
    main()
